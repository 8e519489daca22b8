// mpc_run.h — persistent episode run: K MPC steps of the device-resident
// episode (math_model_tree.py:515-635, heading mode kRotCum) in ONE launch.
//
// Why: a step launched as its own kernel(s) pays, every step, the launch's
// fill and drain (first control loads in flight with nothing to compute, the
// last tiles finishing on a part-idle chip) and the one-block selection
// during which HBM idles: ~6-10 us of a ~37-us config-C step.  In kRotCum
// mode a candidate's rollout needs no start pose (mpc_device.h step_start /
// cum_pose), so step j+1's candidates can stream while step j is still being
// selected; only the final pose transform and the criterion wait for the
// pose.  One launch streams the K steps' tiles back to back:
//
//   unit u = (step j, tile) = (u / T, u % T), T = tiles of 512 candidates per
//   step.  The first block to start selects (run_select_step, one step after
//   the other); every other block streams the units its completer wave claims
//   (one counter, increasing unit order, two units ahead: every claimed unit
//   belongs to a running block, so the lowest unselected unit can always go
//   on — no residency assumption), with 5 waves:
//   - waves 0-3 stream (run_stream_wave): one LDS-DMA control ring per wave
//     that runs ACROSS units (a unit's last steps already issue the next
//     unit's first rows), the step size h speculated from the last head the
//     block knows (+ dt per step, as episode_prepare forms it); at a unit's
//     end a wave parks its lanes' position sums in LDS and goes on — no
//     barrier, no global load, no wait other than its own control rows;
//   - wave 4 completes (run_complete_wave): it waits for step j's published
//     head, turns the parked sums into poses and criteria (recomputing a
//     quarter whose h was mis-speculated — an episode restart reset t — and
//     irregular candidates), reduces the unit to one tagged record and frees
//     the parking slot;
//   - the selector sweeps step j's T records, re-rolls the winner (emit_winner),
//     applies the episode update (episode_advance: finishing logic, operator
//     events, restart, log record, the next step's t and constants) and
//     publishes step j+1's head.
//
// Hand-offs (MI355X_MICROARCH.md "inter-workgroup visibility",
// cdna_hip_programming.md Guideline 16 R2): every handed-off word is an 8-byte
// {data32 << 32 | tag32} granule written by ONE relaxed agent-scope atomic
// store (sc1) and read by relaxed agent-scope atomic loads (sc1); the tag is
// the step index within the call + 1, so a granule validates itself and no
// fence is needed.  The polled words (abort word, head and record granules)
// are zeroed by a memset node before every launch (mpc_episode_run), so a tag
// from an earlier call (or graph replay) never matches.  Inside a block the
// streaming waves and the completer meet only in LDS.  Every wait is bounded:
// on a timeout the waiter sets the abort word (every other wait then gives
// up at once) and chain error 3.
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
#define RUN_STAT(i, v) ((void)0)
#define RUN_TICK() 0ull
#define RUN_ACC(i, v) ((void)0)
#endif

constexpr int kRunRecWords = 4;       // granules per unit record: key hi, key lo, index, pad
constexpr uint32_t kRunSpinLimit = 1u << 18;   // x s_sleep(16) ~1 us: ~0.25 s

// The polled block at the start of the run workspace (zeroed every call).
struct RunCtl {
  uint32_t abort;        // a bounded wait timed out: every wait gives up
  uint32_t claim;        // next unit to hand out (claimed by the completer waves)
  uint32_t role;         // blocks started: the first one selects
  uint32_t pad_[29];
  uint64_t pub[2][kHeadDwords];   // head of step j in pub[j & 1], tag j + 1
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

#ifndef MPC_RUN_WAVES
#define MPC_RUN_WAVES 4   // launch bound of the run kernel (A/B: tools/build_variant.sh)
#endif

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
  if (!last && q < kHeadDwords) granule_store(rc->pub[(j + 1) & 1] + q, tag + 1u, s_head[q]);
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

// Per streaming block: the parking slot (one unit: 4 waves x 64 lanes x two
// candidates' position sums and irregular flags, the h each wave's loop used)
// and the completer's knowledge of the heads (read by the streaming waves
// for the speculation).  LDS only; streaming waves and the completer order
// their accesses with lgkmcnt waits (LDS operations of a wave complete in
// order) and relaxed LDS atomics.
struct RunLds {
  double2 px[kBlock], py[kBlock];   // per streaming lane: (A0, A1), (B0, B1)
  uint32_t bad[kBlock];             // bit c: candidate c irregular
  double ph[kWaves];                // h of each wave's loop
  int32_t cnt;                      // quarters parked in the slot
  int32_t seq;                      // unit index (per block) the slot accepts next
  int32_t jknown;                   // latest step whose head the completer took
  int32_t qn;                       // units claimed for this block so far
  int64_t q[4];                     // unit claimed as the block's k-th in q[k & 3]
  double tring[8];                  // t of step jknown in tring[jknown & 7]
  uint32_t hw[64];                  // the completer's head words (loop words)
};

__device__ __forceinline__ void lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ int32_t lds_load(const int32_t* p) {
  return __hip_atomic_load(const_cast<int32_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Streaming wave (waves 0-3 of blocks 1..): rolls out its quarter (128
// candidates: lane l of wave w holds candidates tile*512 + (64w + l)*2 + {0,1})
// of each of the block's units and parks the sums.  The control ring (kRing
// slots of one step's v and beta rows, kRing-1 steps in flight) continues
// across units; the only waits are the counted vmcnt waits of its own rows
// and, before parking, for the parking slot to be free.
template <int INTEG, bool PL2>
__device__ __forceinline__ void run_stream_wave(RunLds& sh, const double* const* __restrict__ ctl,
                                                int64_t total, int64_t T, int64_t n_cand,
                                                int n_steps, RunCtl* __restrict__ rc,
                                                EpisodeState* __restrict__ S, const Consts& Kc,
                                                double delta_t) {
  constexpr int CPL = 2;
  constexpr int R = kRing;
  constexpr uint32_t kSlot = 2 * 64 * sizeof(double2);   // 2 KiB: v and beta rows
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring0 = __builtin_amdgcn_readfirstlane(lds_addr(&g_ring[wv][0][0][0]));
  auto dst = [&](uint32_t slot) { return ring0 + slot * kSlot; };
  // the block's k-th unit, from the completer's claims (normally long there)
  auto unit_of = [&](int32_t k) -> int64_t {
    for (uint32_t it = 0; lds_load(&sh.qn) <= k; ++it) {
      if ((it & 1023) == 1023 && run_aborted(rc)) return total;
      if (it >= kRunSpinLimit * 8u) {
        if (lane == 0) run_fail(rc, S, 5);
        return total;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    lds_order();
    return sh.q[k & 3];
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
  for (int32_t k = 0; u < total; ++k, u = unit_of(k)) {
    const int64_t j = u / T;
    // step size: from the completer's latest head, + dt per step since
    {
      const int32_t jk = lds_load(&sh.jknown);
      double t = sh.tring[jk & 7];
      for (int64_t q = jk; q < j; ++q) t = t + delta_t;
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
    if (lane == 0) RUN_TL_MIN(j, 0);
#pragma unroll 1
    for (int st = 0; st < n_steps; ++st) {
      issue(true, rv, rb);
      const uint32_t ahead = gi - gc - 1;   // rows in flight behind this one
      if (ahead >= 2)
        wait_vm<2 * (R - 1)>();
      else if (ahead == 1)
        wait_vm<2>();
      else
        wait_vm<0>();
      const uint32_t sl = gc % R;
      rv = g_ring[wv][sl][0][lane];
      rb = g_ring[wv][sl][1][lane];
      ++gc;
      // (the heading itself is not carried: kRotCum rotates (sn, cs))
      double ph0 = 0.0, ph1 = 0.0;
      step_core<INTEG, kRotCum, PL2>(x[0], y[0], ph0, sn[0], cs[0], rv.x, rb.x, Kl, bad[0], &lead);
      step_core<INTEG, kRotCum, PL2>(x[1], y[1], ph1, sn[1], cs[1], rv.y, rb.y, Kl, bad[1], &lead);
    }
    if (lane == 0) RUN_TL_MAX(j, 1);
    // park: wait for the slot (the completer frees it after the previous unit)
    const uint64_t p0t = RUN_TICK();
    if (lds_load(&sh.seq) != k) RUN_ACC(5, 1);
    for (uint32_t it = 0; lds_load(&sh.seq) != k; ++it) {
      if ((it & 1023) == 1023 && run_aborted(rc)) break;
      if (it >= kRunSpinLimit * 8u) {
        if (lane == 0) run_fail(rc, S, 2);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    RUN_ACC(4, RUN_TICK() - p0t);
    sh.px[threadIdx.x] = make_double2(x[0], x[1]);
    sh.py[threadIdx.x] = make_double2(y[0], y[1]);
    sh.bad[threadIdx.x] = (bad[0] ? 1u : 0u) | (bad[1] ? 2u : 0u);
    if (lane == 0) sh.ph[wv] = Kl.h;
    lds_order();   // the quarter's words are in LDS before the count says so
    if (lane == 0)
      __hip_atomic_fetch_add(&sh.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
#ifdef MPC_RUN_STATS
  if (lane == 0)
    for (int q = 0; q < 16; ++q)
      if (st_acc[q]) RUN_STAT(q, st_acc[q]);
#endif
}

// Completer wave (wave 4 of blocks 1..): for each unit of the block, once its
// four quarters are parked and step j's head is published: criteria, the
// unit's (cost, index) minimum, one tagged record; then frees the slot.
template <int INTEG, bool PL2>
__device__ __forceinline__ void run_complete_wave(RunLds& sh, const double* const* __restrict__ ctl,
                                                  int64_t total, int64_t T, int64_t n_cand,
                                                  int n_steps, RunCtl* __restrict__ rc,
                                                  uint64_t* __restrict__ rec,
                                                  EpisodeState* __restrict__ S) {
  constexpr int CPL = 2;
  const int lane = threadIdx.x & 63;
  int64_t jk = 0;
#ifdef MPC_RUN_STATS
  uint64_t st_acc[16] = {0};
#endif
  // claims: units are handed out in increasing order to running blocks only,
  // so the lowest unselected unit's block can always go on; this block's k-th
  // unit is claimed when it starts completing its (k-2)-th
  auto claim = [&](int32_t k) {
    if (lane == 0) {
      const uint32_t c =
          __hip_atomic_fetch_add(&rc->claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sh.q[k & 3] = static_cast<int64_t>(c);
      lds_order();
      lds_store(&sh.qn, k + 1);
    }
  };
  claim(0);
  claim(1);
  for (int32_t k = 0;; ++k) {
    claim(k + 2);
    lds_order();
    const int64_t u = sh.q[k & 3];
    if (u >= total) break;
    const int64_t j = u / T;
    const int64_t tile = u - j * T;
    // all four quarters parked
    const uint64_t c0t = RUN_TICK();
    for (uint32_t it = 0; lds_load(&sh.cnt) != kWaves; ++it) {
      if ((it & 1023) == 1023 && run_aborted(rc)) break;
      if (it >= kRunSpinLimit * 8u) {
        if (lane == 0) run_fail(rc, S, 3);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    lds_order();
    const uint64_t c1t = RUN_TICK();
    RUN_ACC(2, c1t - c0t);
    // step j's head
#ifdef MPC_RUN_NODEP
    if (false) {   // A/B probe only: no dependency on the selection (results invalid)
#else
    if (j != jk) {
#endif
      const uint64_t* g = rc->pub[j & 1];
      const uint32_t tag = static_cast<uint32_t>(j + 1);
      for (uint32_t it = 0; !run_read_words(g, tag, sh.hw); ++it) {
        if (it >= kRunSpinLimit || run_aborted(rc)) {
          if (lane == 0) run_fail(rc, S, 4);
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      lds_order();
      if (lane == 0) sh.tring[j & 7] = run_words_t(sh.hw);
      lds_order();   // t before the step index that points at it
      if (lane == 0) lds_store(&sh.jknown, static_cast<int32_t>(j));
      jk = j;
      RUN_ACC(1, 1);
      RUN_ACC(3, RUN_TICK() - c1t);
    }
    RUN_ACC(0, 1);
    const Consts K = consts_from_words(sh.hw);
    const double* cv = ctl[2 * j];
    const double* cb = ctl[2 * j + 1];
    uint64_t best_k = ~0ull;
    int64_t best_i = INT64_MAX;
#pragma unroll 1
    for (int w = 0; w < kWaves; ++w) {
      const int tq = w * 64 + lane;
      const double2 px = sh.px[tq], py = sh.py[tq];
      const uint32_t bb = sh.bad[tq];
      const double hq = sh.ph[w];
      const int64_t c0 = tile * (kBlock * CPL) + tq * CPL;
      const int64_t cl = c0 < n_cand ? c0 : n_cand - CPL;
      const double ax[CPL] = {px.x, px.y}, ay[CPL] = {py.x, py.y};
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        double cst;
#ifdef MPC_RUN_NODEP
        if (false) {
#else
        if (hq != K.h) {   // mis-speculated step size (an episode restart reset t)
#endif
          cst = rollout_candidate_l<INTEG, kRotCum, PL2>(K, cv, cb, n_cand, cl + c, n_steps,
                                                         nullptr);
        } else if (bb & (1u << c)) {   // irregular candidate: the safe recurrence
          double xx = K.x, yy = K.y, ph = K.phi;
          for (int sr = 0; sr < n_steps; ++sr)
            step_safe<INTEG>(xx, yy, ph, cv[sr * n_cand + cl + c], cb[sr * n_cand + cl + c], K);
          cst = cost(xx, yy, K);
        } else {
          double xx, yy;
          cum_pose(K, ax[c], ay[c], xx, yy);
          cst = cost(xx, yy, K);
        }
        const uint64_t kk = cost_key(cst);
        if (c0 + c < n_cand && rec_less(kk, c0 + c, best_k, best_i)) {
          best_k = kk;
          best_i = c0 + c;
        }
      }
    }
    wave_argmin(best_k, best_i);
    if (lane == 0) {
      const uint32_t tag = static_cast<uint32_t>(j + 1);
      uint64_t* r = rec + ((j & 1) * T + tile) * kRunRecWords;
      granule_store(r, tag, static_cast<uint32_t>(best_k >> 32));
      granule_store(r + 1, tag, static_cast<uint32_t>(best_k));
      granule_store(r + 2, tag, static_cast<uint32_t>(best_i));   // < 2^31 (host check)
      RUN_TL_MAX(j, 2);
    }
    // free the slot: its words are read (lgkmcnt) before the next unit may write
    lds_order();
    if (lane == 0) {
      lds_store(&sh.cnt, 0);
      lds_order();
      lds_store(&sh.seq, k + 1);
    }
  }
#ifdef MPC_RUN_STATS
  if (lane == 0)
    for (int q = 0; q < 16; ++q)
      if (st_acc[q]) RUN_STAT(q, st_acc[q]);
#endif
}

constexpr int kRunThreads = kBlock + 64;   // 4 streaming waves + the completer
#ifndef MPC_RUN_WAVES
#define MPC_RUN_WAVES 5   // waves per SIMD: 4 blocks of 5 waves per CU
#endif

// ctl: device array [k_steps][2] of the steps' control SoA pointers (v, beta).
// rec: [2][T][kRunRecWords] record granules (step j in half j & 1).
// out: step k_steps-1's winner; every other step's re-roll goes to scratch.
// clock: optional [k_steps] s_memrealtime (100 MHz) when step j was completed.
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
  const int wv = threadIdx.x >> 6;
  // Roles: the first block to start selects (so the selector is a running
  // block whatever the dispatch order); the others stream and complete.
  __shared__ RunLds sh;
  __shared__ uint32_t s_role;
  if (threadIdx.x == 0)
    s_role = __hip_atomic_fetch_add(&rc->role, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (wv == kWaves) {   // the head of the call's first step (S->h, written before the launch)
    const int q = threadIdx.x & 63;
    if (run_loop_word(q)) sh.hw[q] = reinterpret_cast<const uint32_t*>(&S->h)[q];
    if (q == 0) {
      sh.tring[0] = S->h.t;
      sh.jknown = 0;
      sh.cnt = 0;
      sh.seq = 0;
      sh.qn = 0;
    }
  }
  __syncthreads();   // the only barrier of a streaming block
  if (s_role == 0u) {
    // the selector runs on waves 0-3; a wave that has ended no longer counts
    // at the block's barriers
    if (wv >= kWaves) return;
    // The host picked PL2 from cfg; a state reset with another wheelbase form
    // would be rolled out with the wrong dphi form: flag it (as the chain does).
    if (threadIdx.x == 0 && (S->h.K.L_pow2 != 0) != PL2) S->chain_error = 2u;
    if (threadIdx.x == 0) g_run_cfg = ecfg;
    if (threadIdx.x < kHeadDwords)
      g_run_head[threadIdx.x] = reinterpret_cast<const uint32_t*>(&S->h)[threadIdx.x];
    __syncthreads();
    for (int j = 0; j < k_steps; ++j)
      run_select_step<INTEG>(j, S, ctl[2 * j], ctl[2 * j + 1], k_steps, n_cand, n_steps,
                             index_base, rc, rec, T, j + 1 == k_steps ? out : scratch, log, cap,
                             clock);
    return;
  }
  if (wv < kWaves) {
    const Consts Kc = consts_from_words(sh.hw);   // wheelbase terms (h set per unit)
    run_stream_wave<INTEG, PL2>(sh, ctl, total, T, n_cand, n_steps, rc, S, Kc, ecfg.delta_t);
  } else {
    run_complete_wave<INTEG, PL2>(sh, ctl, total, T, n_cand, n_steps, rc, rec, S);
  }
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
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    cache[dev] = static_cast<int64_t>(per_cu) * cus;
  }
  // one block selects; at least one streams
  return std::max<int64_t>(2, std::min(total_units + 1, cache[dev]));
}

}  // namespace mpc
