// mpc_run.h — persistent episode run: K MPC steps of the one-GPU chained
// episode (math_model_tree.py:515-635 around predictive_control :278-496,
// heading mode kRotCum) in ONE launch (mpc_episode_run).
//
// Why: one chained launch per step (k_episode_chain) pays per step a kernel
// boundary, the launch's ramp and its 1.27-round tile tail (the last ~420
// tiles of config C stream at ~2.8 TB/s for their last ~12 us), and the
// captured sequence needs a closing flush launch.  In kRotCum mode a
// candidate's rollout needs no start pose (mpc_device.h step_start /
// cum_pose): step j+1's tiles can stream while step j's last tiles finish and
// step j is being selected; only the final pose transform and the criterion
// wait for the pose.
//
//   unit u = (step j, tile) = (u / T, u % T), T = tiles of 512 candidates.
//   Block 0 is the SELECTOR: it publishes step 0's constants, then for j =
//   0..K-1 polls step j's T tagged records, reduces them, re-rolls the winner
//   and applies the episode update (finalize_block: the chained step's block
//   0 code, early publication included) — which publishes step j+1's
//   constants (epoch e0 + j + 1) or, after the last step, clears the tags.
//   Blocks 1.. CLAIM units in increasing order from one counter (thread 0,
//   the next claim in flight during the current unit) and run the chained
//   step's tile body on each (speculated step size, the published constants
//   at the end, a tagged record into part[j & 1][tile]).
//
// Deadlock freedom: a unit is claimed only by a running block, and a block
// holding a unit of step j waits only for step j's constants, which need only
// the records of step j-1 — every one of them claimed earlier, by running
// blocks whose own waits are for steps < j (induction over j; step 0's
// constants are published at once).  So any grid size is safe, resident or
// not (round 2's persistent run assigned units by blockIdx and deadlocked
// once the occupancy API over-promised; it also kept pending quarters in
// registers: 152 VGPRs, 3 waves per SIMD — this body is the chained kernel's,
// 5 waves).  Every wait is bounded (chain error 1 in a tile, 3 in the
// selector) and a timed-out selector still publishes, so the launch drains.
//
// Hand-offs: the records are 16-B tagged granules (store_tagged_rec: both 8-B
// halves carry rec_tag(epoch)), polled by the selector with `sc1` loads and
// zeroed by it with coherent stores one step later (before the slot's next
// writer can have seen the constants that let it store).  The published
// constants are mpc_episode.h's chain_pub words.  The claim counter is reset
// by the last block to leave, so between launches the workspace is all zero
// (graph replays repeat their epochs safely).
#pragma once

#include "mpc_episode.h"

namespace mpc {

constexpr int kRunMaxSteps = 64;   // steps per launch (the host splits longer runs)

#ifdef MPC_RUN_STATS
// Debug builds only (tools/build_variant.sh-style -DMPC_RUN_STATS): 100-MHz
// stamps per step of the last launch, read by mpc_debug_run_stats:
//   0 selector step start, 1 records complete, 2 step done (selector),
//   3 first unit start (min), 4 last loop end (max), 5 last wait end (max),
//   6 last record stored (max), 7 units that waited
__device__ unsigned long long g_run_tl[kRunMaxSteps][8];
#define RUN_T() __builtin_amdgcn_s_memrealtime()
#define RUN_SET(j, f) (g_run_tl[(j)][(f)] = RUN_T())
#define RUN_MIN(j, f) atomicMin(&g_run_tl[(j)][(f)], RUN_T())
#define RUN_MAX(j, f) atomicMax(&g_run_tl[(j)][(f)], RUN_T())
#define RUN_ADD(j, f) atomicAdd(&g_run_tl[(j)][(f)], 1ull)
#else
#define RUN_SET(j, f) ((void)0)
#define RUN_MIN(j, f) ((void)0)
#define RUN_MAX(j, f) ((void)0)
#define RUN_ADD(j, f) ((void)0)
#endif

// The step's control rows, by value in the kernel arguments.
struct RunCtl {
  const double* v[kRunMaxSteps];
  const double* b[kRunMaxSteps];
};

// The run's arguments live in the kernarg segment (constant address space):
// indexed through such a pointer they stay scalar loads.
typedef const __attribute__((address_space(4))) RunCtl* RunCtlPtr;

// The polled words at the start of the run workspace, then part[2][T].
struct RunHdr {
  uint32_t claim;    // next unit to hand out
  uint32_t exited;   // tile blocks that have left
  uint32_t pad_[62];
};
static_assert(sizeof(RunHdr) == 256, "records start 256 B in");

__host__ __device__ inline size_t run_workspace_bytes(int64_t tiles) {
  return sizeof(RunHdr) + 2 * static_cast<size_t>(tiles) * sizeof(Rec);
}

// Selector, all threads: zero the records of slot `z` (the previous step's,
// consumed), then poll step e's T records in `p` until every one carries
// rec_tag(e) (bounded: chain error 3), leaving each thread's lexicographic
// (cost key, local index) minimum of its records in (k, i).  Returns false on
// a timeout.
__device__ bool run_poll_records(const Rec* __restrict__ p, Rec* __restrict__ z, int T, uint32_t e,
                                 uint64_t& k, int64_t& i) {
  k = ~0ull;
  i = INT64_MAX;
  if (z) {
    for (int q = threadIdx.x; q < T; q += kBlock) {
      uint64_t* h = reinterpret_cast<uint64_t*>(&z[q]);
      __hip_atomic_store(h, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(h + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const uint32_t tag = rec_tag(e);
  const uint32_t deadline = wall_deadline(kChainWaitTicks);
  for (int base = 0; base < T; base += 8 * kBlock) {
    uint32_t off[8];
    u64x2 r[8];
    const int n = T - base < 8 * kBlock ? T - base : 8 * kBlock;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int pi = threadIdx.x + q * kBlock;
      off[q] = static_cast<uint32_t>(pi < n ? pi : n - 1) * sizeof(Rec);
    }
    for (uint32_t it = 0;; ++it) {
      load8_rec_sc1_sbase(p + base, off, r);
      bool ok = true;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (threadIdx.x + q * kBlock < n) ok = ok && tagged_rec_fresh(r[q], tag);
      if (__syncthreads_and(ok)) break;
      if ((it & 15) == 15 && block_wall_passed(deadline)) return false;   // (uniform)
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (threadIdx.x + q * kBlock < n) {
        const uint32_t lo = tagged_rec_index(r[q]);
        const int64_t idx = lo == 0xffffffffu ? INT64_MAX : static_cast<int64_t>(lo);
        const uint64_t key = tagged_rec_key(r[q]);
        if (rec_less(key, idx, k, i)) {
          k = key;
          i = idx;
        }
      }
    }
  }
  return true;
}

// Tile blocks: claim units in order and run the chained step's tile body on
// each (chain_tiles, mpc_episode.h, for one tile of step j with epoch e0 + j).
template <bool PL2, bool TILED>
__device__ __forceinline__ void run_tiles(EpisodeState* __restrict__ S, uint32_t e0,
                                          RunCtlPtr ctl, int K, int64_t n_cand, int n_steps,
                                          RunHdr* __restrict__ hdr, Rec* __restrict__ part,
                                          int T, const mpc_episode_config_t& ecfg) {
  constexpr int INTEG = MPC_INTEG_RECT, ROT = kRotCum;
  constexpr int CPL = 2;
  __shared__ __attribute__((aligned(16))) uint32_t s_w[kPubWords];
  __shared__ uint32_t s_tag[kPubWords];
  __shared__ int s_final, s_untagged;
  __shared__ uint32_t s_claim;
  static_assert(offsetof(Consts, x) == 0 && alignof(Consts) <= 16, "Consts over s_w");
  const Consts& Kc = *reinterpret_cast<const Consts*>(s_w);
  const uint32_t total = static_cast<uint32_t>(K) * static_cast<uint32_t>(T);
  if (threadIdx.x == 0)
    s_claim = __hip_atomic_fetch_add(&hdr->claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  uint32_t u = __builtin_amdgcn_readfirstlane(s_claim);
  const int32_t n32 = static_cast<int32_t>(n_cand);
  while (u < total) {
    // the next claim, in flight during this unit (thread 0; read at its end)
    uint32_t nxt = 0;
    if (threadIdx.x == 0)
      nxt = __hip_atomic_fetch_add(&hdr->claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int j = static_cast<int>(u / static_cast<uint32_t>(T));
    const int32_t tile = static_cast<int32_t>(u - static_cast<uint32_t>(j) * T);
    const uint32_t epoch = e0 + static_cast<uint32_t>(j);
    const double* v = ctl->v[j];
    const double* b = ctl->b[j];
    if (threadIdx.x == 0) RUN_MIN(j, 3);
    Consts Kl;
    bool waited = false;
    auto pre0 = [&]() {
      if (threadIdx.x < 64) {
        bool fin = true, untagged = false;
        if (j > 0) {
          fin = chain_read(S, epoch, s_w, s_tag);
          // a word never published in this launch (tag 0: the previous run
          // cleared them) carries no loop constants (the wheelbase terms)
          untagged = __ballot(threadIdx.x < kPubWords && s_tag[threadIdx.x] == 0u) != 0;
        } else if (threadIdx.x < kConstsWords) {
          // step 0: the head as the previous launch (or reset) left it — final,
          // and not updated before every step-0 record is in
          s_w[threadIdx.x] = reinterpret_cast<const uint32_t*>(&S->h.K)[threadIdx.x];
        }
        if (threadIdx.x == 0) {
          s_final = fin;
          s_untagged = untagged;
        }
      }
      __syncthreads();
      Kl = consts_from_words(s_w);
      if (s_final) return;
      // speculate h from the published t: one or two steps behind (+ dt each,
      // as episode_prepare forms it) or this step's; otherwise — or while any
      // word is untagged (epoch - 2 would match tag 0 at step 1) — NaN: the
      // loop reruns with the final constants
      const uint32_t g0 = __builtin_amdgcn_readfirstlane(s_tag[kConstsWords]);
      const uint32_t g1 = __builtin_amdgcn_readfirstlane(s_tag[kConstsWords + 1]);
      const uint64_t tb =
          (static_cast<uint64_t>(static_cast<uint32_t>(
               __builtin_amdgcn_readfirstlane(s_w[kConstsWords + 1]))) << 32) |
          static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(s_w[kConstsWords]));
      double t = __longlong_as_double(static_cast<long long>(tb));
      if (g0 == g1 && g0 == epoch - 1u)
        t = t + ecfg.delta_t;
      else if (g0 == g1 && g0 == epoch - 2u)
        t = (t + ecfg.delta_t) + ecfg.delta_t;
      else if (!(g0 == g1 && g0 == epoch))
        t = __builtin_nan("");
      if (s_untagged) t = __builtin_nan("");
      Kl.h = (t + ecfg.delta_t) - t;
    };
    uint64_t w_pre = 0;
    bool pre_issued = false;
    auto mid = [&]() {
      if (waited || pre_issued || s_final) return;
      pre_issued = true;
      if (threadIdx.x < kPubWords)
        w_pre = __hip_atomic_load(&S->chain_pub[threadIdx.x], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    };
    auto wait = [&]() {
      if (waited) return;
      waited = true;
      if (threadIdx.x == 0) RUN_MAX(j, 4);
      __syncthreads();
      if (!s_final) {
        if (threadIdx.x == 0) RUN_ADD(j, 7);
        if (threadIdx.x < 64) {
          bool fin = false;
          if (pre_issued) {
            const bool ok = threadIdx.x >= kPubWords || static_cast<uint32_t>(w_pre) == epoch;
            fin = __ballot(!ok) == 0;
            if (fin && threadIdx.x < kPubWords) s_w[threadIdx.x] = static_cast<uint32_t>(w_pre >> 32);
          }
          if (!fin) {
            const uint32_t deadline = wall_deadline(kChainWaitTicks);
            const int q = threadIdx.x;
            uint64_t* const pw = &S->chain_pub[q < kPubWords ? q : 0];
            auto ld = [&]() {
              return __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
            auto here = [&](uint64_t w) {
              return __ballot(q < kPubWords && static_cast<uint32_t>(w) != epoch) == 0;
            };
            uint64_t a = ld(), bb = 0, got = 0;
            for (;;) {
              __builtin_amdgcn_s_sleep(2);
              bb = ld();
              if (here(a)) { got = a; fin = true; break; }
              if (wall_passed(deadline)) break;
              __builtin_amdgcn_s_sleep(2);
              a = ld();
              if (here(bb)) { got = bb; fin = true; break; }
              if (wall_passed(deadline)) break;
            }
            if (fin && q < kPubWords) s_w[q] = static_cast<uint32_t>(got >> 32);
          }
          if (!fin && threadIdx.x == 0) S->chain_error = 1u;
        }
        __syncthreads();
      }
      if (threadIdx.x == 0) RUN_MAX(j, 5);
    };
    const int32_t c0 = tile * (kBlock * CPL) + static_cast<int32_t>(threadIdx.x) * CPL;
    const int32_t cl = min(c0, n32 - CPL);
    double cst[CPL];
    const int64_t tb0 = TILED ? static_cast<int64_t>(tile) * (2 * MPC_TILE) * n_steps : 0;
    rollout_lane_glds_k<INTEG, ROT, PL2, decltype(wait), decltype(pre0), decltype(mid), false>(
        Kc, Kl, v + tb0, b + tb0, TILED ? 2 * MPC_TILE : n_cand,
        TILED ? cl - tile * MPC_TILE : cl, n_steps, cst, wait, pre0, mid);
    uint64_t best_k = ~0ull;
    int64_t best_i = INT64_MAX;
    if (c0 < n32) {
#pragma unroll
      for (int jj = 0; jj < CPL; ++jj) {
        const uint64_t kk = cost_key_nonneg(cst[jj]);
        if (kk < best_k) {
          best_k = kk;
          best_i = c0 + jj;
        }
      }
    }
    block_argmin<true>(best_k, best_i);
    if (threadIdx.x == 0) {
      store_tagged_rec(&part[static_cast<size_t>(j & 1) * T + tile], best_k, best_i, epoch);
      RUN_MAX(j, 6);
      s_claim = nxt;
    }
    __syncthreads();   // s_claim; s_w / the ring reused by the next unit
    u = __builtin_amdgcn_readfirstlane(s_claim);
  }
  // the last block to leave resets the counter (every block made its last
  // claim before leaving)
  if (threadIdx.x == 0) {
    const uint32_t gone =
        __hip_atomic_fetch_add(&hdr->exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (gone == gridDim.x - 1) {
      __hip_atomic_store(&hdr->claim, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&hdr->exited, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// All arguments in ONE by-value struct, read through the kernarg segment
// pointer: the per-step control pointers are indexed by a runtime step, and a
// by-value array indexed so is copied to scratch (320 B per lane measured).
struct RunArgs {
  EpisodeState* S;
  void* ws;
  mpc_result_t* out;
  mpc_episode_log_t* log;
  int64_t n_cand, index_base;
  uint32_t e0;
  int K, n_steps, T, cap, pad_;
  mpc_episode_config_t ecfg;
  RunCtl ctl;
};

// Block 0, one step: complete step j (poll its records, reduce, re-roll the
// winner, update the episode, publish step j+1's constants — or, after the
// last step, clear the tags).  Every argument is re-read from the kernarg
// segment here (the caller launders the pointer per step): held across the
// step loop they spilled to scratch (320 B per lane), and the reloads sat on
// the selection's serial chain.
template <bool TILED>
__device__ __attribute__((noinline)) void run_select_step(uint64_t args_at, int j_in) {
  // (a call passes its arguments in VGPRs: the step index and the kernarg
  // address made uniform again, so that the head's constants and every
  // pointer read from the arguments stay scalar)
  const int j = __builtin_amdgcn_readfirstlane(j_in);
  const uint64_t at =
      (static_cast<uint64_t>(static_cast<uint32_t>(
           __builtin_amdgcn_readfirstlane(static_cast<int>(args_at >> 32)))) << 32) |
      static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(args_at)));
  const __attribute__((address_space(4))) RunArgs& a =
      *(const __attribute__((address_space(4))) RunArgs*)at;
  EpisodeState* S = a.S;
  const int T = a.T, K = a.K;
  Rec* part = reinterpret_cast<Rec*>(static_cast<char*>(a.ws) + sizeof(RunHdr));
  const uint32_t e = a.e0 + static_cast<uint32_t>(j);
  const Rec* pj = part + static_cast<size_t>(j & 1) * T;
  Rec* pz = j > 0 ? part + static_cast<size_t>((j - 1) & 1) * T : nullptr;
  bool ok = true;
  if (threadIdx.x == 0) RUN_SET(j, 0);
  auto src = [&](uint64_t& k, int64_t& i) {
    ok = run_poll_records(pj, pz, T, e, k, i);
    if (threadIdx.x == 0) RUN_SET(j, 1);
  };
  const Consts Kp = S->h.K;
  const uint32_t next = j + 1 < K ? e + 1u : 0u;   // 0: the run ends the chain
  const EpisodeHook hook{&S->h, a.log, a.cap, S->chain_pub, kPubWords, next, &S->chain_error};
  const mpc_episode_config_t& ecfg = *(const mpc_episode_config_t*)&a.ecfg;
  finalize_block<MPC_INTEG_RECT, kRotCum, true, kBlock, false, false, TILED>(
      nullptr, T, Kp, a.ctl.v[j], a.ctl.b[j], a.n_cand, a.n_steps, a.index_base,
      S->h.incumbent, a.out, ecfg, hook, ring_lds(), src);
  if (!ok && threadIdx.x == 0) S->chain_error = 3u;
  if (threadIdx.x == 0) RUN_SET(j, 2);
}

template <bool PL2, bool TILED>
__global__ __launch_bounds__(kBlock, MPC_CHAIN_FIN_WAVES) void k_episode_run(RunArgs args) {
  typedef const __attribute__((address_space(4))) RunArgs* ArgPtr;
  ArgPtr ap = (ArgPtr)__builtin_amdgcn_kernarg_segment_ptr();
  if (blockIdx.x == 0) {
    // the selector: step 0's constants are the head as reset / last updated
    chain_publish(ap->S, ap->e0);
    if (threadIdx.x == 0 && (ap->S->h.K.L_pow2 != 0) != PL2) ap->S->chain_error = 2u;
    const int K = ap->K;
    for (int j = 0; j < K; ++j) {
      run_select_step<TILED>(reinterpret_cast<uint64_t>(ap), j);
      __syncthreads();   // the head's stores before the next step's staging loads
    }
    // the last step's records, consumed: zero them (the workspace is all zero
    // between launches)
    ArgPtr al = ap;
    asm volatile("" : "+s"(al));
    const int T = al->T;
    Rec* pz = reinterpret_cast<Rec*>(static_cast<char*>(al->ws) + sizeof(RunHdr)) +
              static_cast<size_t>((K - 1) & 1) * T;
    for (int q = threadIdx.x; q < T; q += kBlock) {
      uint64_t* h = reinterpret_cast<uint64_t*>(&pz[q]);
      __hip_atomic_store(h, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(h + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const __attribute__((address_space(4))) RunArgs& a = *ap;
  RunHdr* hdr = static_cast<RunHdr*>(a.ws);
  Rec* part = reinterpret_cast<Rec*>(static_cast<char*>(a.ws) + sizeof(RunHdr));
  run_tiles<PL2, TILED>(a.S, a.e0, &a.ctl, a.K, a.n_cand, a.n_steps, hdr, part, a.T, args.ecfg);
}

}  // namespace mpc
