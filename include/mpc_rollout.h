/*
 * mpc_rollout.h — C ABI of the MI355X-native MPC candidate expansion.
 *
 * Drop-in boundary for ShittyWizard/DiplomJourney's hot path:
 * the body of `predictive_control` in math_model_tree.py:278-362 — roll the
 * bicycle-kinematic step (math_model_tree.py:69-115) forward over an N-step
 * horizon for every candidate control sequence, score the layer-N state with
 * `control_criterion` (:56-87) and keep the first strict minimum (:351-359).
 *
 * The reference has no FFI (it is pure Python); these entry points are what
 * its Python host binds through ctypes.  Plain pointers and
 * sizes only: every device buffer is owned by the caller, borrowed for the
 * call, never retained.  No function throws or aborts; all return an int
 * status (MPC_OK = 0, negative on error, see mpc_strerror).
 *
 * Data layout in HBM (SoA, step-major, fp64):
 *   v_sc[s * n_cand + c], beta_sc[s * n_cand + c]   s < n_steps, c < n_cand
 * Candidate c's global index is index_base + c (contiguous shards across GPUs).
 *
 * The fast ("aligned") path: n_cand even, v_sc and beta_sc 16-B aligned, and
 * rows of fewer than 2^28 candidates (the LDS-DMA control loads address a row
 * as an SGPR base plus a 32-bit lane byte offset).  Other shapes run the one-
 * candidate-per-lane kernel (same results, several times slower) in the
 * one-shot and two-launch entries; the chained and exchange entries, which
 * exist only on the aligned path, return MPC_ERR_UNSUPPORTED.
 */
#ifndef DIPLOMJOURNEY_AMD_MPC_ROLLOUT_H
#define DIPLOMJOURNEY_AMD_MPC_ROLLOUT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* mpc_stream_t; /* == hipStream_t */

#define MPC_MAX_STEPS 32

enum {
  MPC_OK = 0,
  MPC_ERR_ARG = -1,         /* bad size / null pointer / n_steps out of range   */
  MPC_ERR_WORKSPACE = -2,   /* ws_bytes < required                              */
  MPC_ERR_HIP = -3,         /* a HIP runtime call failed (launch, copy)         */
  MPC_ERR_UNSUPPORTED = -4  /* e.g. integrator id unknown                       */
};

/* How the constant integrand of each quad() call is integrated.
 * QK21: bit-faithful emulation of scipy.integrate.quad -> QUADPACK qk21 on a
 *       constant integrand (math_model_tree.py:91-96; SURVEY Fact 4).
 * RECT: the same integrals of the constant integrands evaluated directly:
 *       dphi = ((v / L) * h) * tan(beta), x' = fma(v * h, cos(phi'), x),
 *       h = t_b - t_a (exact integral, fewer roundings; mpc_device.h).   */
enum { MPC_INTEG_QK21 = 0, MPC_INTEG_RECT = 1 };

/* Flag OR'ed into every `integrator` argument: carry (sin, cos) of the heading
 * along the rollout and rotate it by each step's increment dphi instead of
 * evaluating sin/cos of the new heading (math_model_tree.py:113-114) with a
 * full range reduction.  Same mathematics, different rounding (a few ulp on
 * the heading's sin/cos after N steps); ~40% fewer VALU instructions per
 * candidate-step.  Candidates with an increment |dphi| > 0.2 (or |beta| > 1.1)
 * are recomputed with direct evaluation. */
#define MPC_HEADING_ROTATE 0x100
/* RECT only: the rotation recurrence started from the identity (sin, cos) =
 * (0, 1) and position sums (A, B) = (0, 0) — A = sum v h cos(Phi_k),
 * B = sum v h sin(Phi_k) over the heading increments Phi_k since the start —
 * and the start pose applied last: x = x0 + (c0 A - s0 B), y = y0 + (s0 A +
 * c0 B).  Same work per step as MPC_HEADING_ROTATE, other roundings (ulps);
 * a candidate's rollout then needs no start pose, which lets a chained
 * episode step (mpc_episode_chain_step) roll out step k while step k-1 is
 * still being selected.  Irregular candidates as above. */
#define MPC_HEADING_CUMULATIVE 0x200
/* Control layout flag, OR'ed into `integrator` of the chained one-GPU and P2P
 * episode entries and their flush (mpc_episode_chain_step,
 * mpc_episode_finalize, mpc_episode_p2p_step, mpc_episode_p2p_flush): the
 * candidates are TILED instead of step-major SoA — tile t of 512 consecutive
 * candidates holds, for each step s, its 512 v values then its 512 beta values,
 *   v    (c, s) = base[(c / 512) * 1024 * n_steps + s * 1024 + c % 512]
 *   beta (c, s) = the same + 512
 * (mpc_tiled_index; allocation: ceil(n_cand / 512) * 1024 * n_steps doubles).
 * The caller passes v_sc = base and beta_sc = base + 512.  One tile's whole
 * horizon is one contiguous 8-KiB-per-step run, so a tile block's control
 * stream stays within a few DRAM pages instead of striding by 8 * n_cand
 * bytes per step (measured, tools/micro/layout_probe.hip: 6.31 vs 6.14 TB/s at
 * 1e6 x N = 10).  mpc_sample_controls_tiled writes this layout. */
#define MPC_LAYOUT_TILED 0x400
#define MPC_TILE 512

/* One MPC problem (one robot at one MPC step). */
typedef struct mpc_problem {
  double x, y, phi;   /* initial_coordinates, math_model_tree.py:294            */
  double x_t, y_t;    /* target globals read by the cost, :56-66                */
  double x_0, y_0;    /* line-origin globals, :57-61                            */
  double L;           /* wheelbase, config.py:6 (v_phi, :77-78)                 */
  double t_a, t_b;    /* quad limits [t, t + delta_t], :99-108 (t advanced :302) */
} mpc_problem_t;

/* The selected candidate.  `found` == 0 means no candidate beat `incumbent`
 * (strict <, :351): the caller keeps its stale trajectory. */
/* One rank's best candidate of a sharded MPC step, as the multi-GPU exchange
 * gathers it: the arg-min's (cost, global index) and the candidate's
 * controls, so that whichever rank holds the global winner, every rank can
 * re-roll it (mpc_episode_exchange_step).  536 B. */
typedef struct mpc_candidate {
  double cost;                      /* +inf when the shard has no finite cost  */
  int64_t index;                    /* global index, -1 when none              */
  int32_t n_steps, reserved_;
  double v[MPC_MAX_STEPS], beta[MPC_MAX_STEPS];   /* its controls, per step  */
} mpc_candidate_t;

typedef struct mpc_result {
  double cost;                      /* control_criterion of the winner         */
  int64_t index;                    /* global index, -1 when no finite cost    */
  int32_t found;                    /* cost < incumbent                        */
  int32_t n_steps;
  double v, beta;                   /* winner's step-0 control (:357-358)      */
  double traj[MPC_MAX_STEPS][3];    /* (x, y, phi) after each step (:353-356)  */
} mpc_result_t;

const char* mpc_version(void);
const char* mpc_strerror(int status);

/* Workspace for mpc_rollout_argmin (per-block partial arg-min records). */
size_t mpc_workspace_bytes(int64_t n_cand, int32_t n_steps);

/*
 * Expansion + arg-min of one problem: replaces math_model_tree.py:295-360
 * (CoordinateTree fill + layer loops + strict-< scan) for n_steps layers.
 *   p           host pointer, read during the call only
 *   states_out  optional device buffer [n_steps][3][n_cand] (x, y, phi of every
 *               candidate after every step: the CoordinateTree payload); NULL
 *               skips it (the benchmark path)
 *   out         device pointer to one mpc_result_t, written on `stream`
 * Ties resolve to the lowest global index, NaN costs never win.
 */
int mpc_rollout_argmin(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                       int64_t n_cand, int32_t n_steps, int64_t index_base, double incumbent,
                       int32_t integrator, double* states_out, void* ws, size_t ws_bytes,
                       mpc_result_t* out, mpc_stream_t stream);

/* The two launches mpc_rollout_argmin enqueues, exposed separately so a
 * caller can time the streaming kernel alone (bench.py) or interleave other
 * work (an exchange) between them.  Same arguments and semantics:
 *   phase 1  mpc_rollout_partials: rollout + cost + per-block arg-min records
 *            into ws (the HBM-streaming kernel)
 *   phase 2  mpc_rollout_finalize: block records -> winner, winner re-rolled
 *            into *out
 * states_out is only accepted by phase 1 (NULL in phase 2's contract). */
int mpc_rollout_partials(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                         int64_t n_cand, int32_t n_steps, int32_t integrator, double* states_out,
                         void* ws, size_t ws_bytes, mpc_stream_t stream);
int mpc_rollout_finalize(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                         int64_t n_cand, int32_t n_steps, int64_t index_base, double incumbent,
                         int32_t integrator, int32_t with_states, void* ws, size_t ws_bytes,
                         mpc_result_t* out, mpc_stream_t stream);

/* Batched robots: R problems, robot r owns columns
 * [r*cand_per_problem, (r+1)*cand_per_problem) of the [n_steps][R*cand] SoA.
 * problems / incumbents (nullable => +inf) / out are device arrays of R.
 * Result indices are local to the robot (0 .. cand_per_problem-1). */
size_t mpc_batched_workspace_bytes(int32_t n_problems, int64_t cand_per_problem, int32_t n_steps);
int mpc_rollout_argmin_batched(const mpc_problem_t* problems, const double* incumbents,
                               int32_t n_problems, const double* v_sc, const double* beta_sc,
                               int64_t cand_per_problem, int32_t n_steps, int32_t integrator,
                               void* ws, size_t ws_bytes, mpc_result_t* out, mpc_stream_t stream);

/* Multi-GPU exchange, device side: pick the lexicographic (cost, index) min
 * of n gathered per-rank results (all_gather output) into *out — the
 * all-reduce(min+index) of SURVEY §8e.  `found` is recomputed against
 * `incumbent`.  Device pointers. */
int mpc_select_winner(const mpc_result_t* results, int32_t n, double incumbent,
                      mpc_result_t* out, mpc_stream_t stream);

/* Measurement probe (not a reference operation): the streaming kernel's
 * memory side alone over the same controls — same grid, tiles and LDS-DMA
 * control ring, no rollout arithmetic — so its duration is the read-only
 * HBM ceiling of the rollout's own access pattern at this size (bench.py's
 * roofline `stream_ceiling`).  Aligned path only (n_cand even, 16-B aligned
 * controls); sink: device scratch of >= 2048 * 256 * 8 bytes (almost never
 * written). */
int mpc_stream_probe(const double* v_sc, const double* beta_sc, int64_t n_cand,
                     int32_t n_steps, void* sink, size_t sink_bytes, mpc_stream_t stream);
/* The same probe over TILED controls (MPC_LAYOUT_TILED; tiles = the tiled
 * buffer's base): the ceiling of the chained kernel's tiled access pattern. */
int mpc_stream_probe_tiled(const double* tiles, int64_t n_cand, int32_t n_steps, void* sink,
                           size_t sink_bytes, mpc_stream_t stream);

/* Verification probe (not a reference operation): the hardware reciprocal
 * estimate the rollout's steering tangent starts from (v_rcp_f64, before its
 * Newton step), r[i] for q[i], device arrays of n doubles.  A host build of
 * the kernel's arithmetic (tests/replica_harness.cpp) installs these values to
 * reproduce the device's bits: the estimate is not an IEEE operation. */
int mpc_rcp_estimate(const double* q, double* r, int64_t n, mpc_stream_t stream);

/* Synthetic candidate generator.  Candidate with
 * global index g = index_base + c:
 *   if const_prefix && g < n_v*n_beta: constant sequence u = (v_grid[g / n_beta],
 *      beta_grid[g % n_beta]) at every step (the reference's enumeration, :311-317)
 *   else step s uses grid entry k = (hi32(splitmix64(seed ^ (s << 40) ^ g)) * n) >> 32
 *      with n = n_v*n_beta (multiply-shift map of the hash onto [0, n))
 * v_grid / beta_grid are device arrays; outputs are written SoA with leading
 * dimension ld >= n_cand: v_sc[s * ld + c] (ld = R*cand lets one call fill one
 * robot's columns of the batched layout). */
int mpc_sample_controls(const double* v_grid, int32_t n_v, const double* beta_grid,
                        int32_t n_beta, int64_t n_cand, int32_t n_steps, uint64_t seed,
                        int64_t index_base, int32_t const_prefix, double* v_sc,
                        double* beta_sc, int64_t ld, mpc_stream_t stream);
/* The same candidates written in the TILED layout (MPC_LAYOUT_TILED) into
 * tiles[ceil(n_cand / 512) * 1024 * n_steps] (16-B aligned, n_cand even); the
 * last tile's padding slots hold the generator's values of the global indices
 * that follow (they are never read as candidates). */
int mpc_sample_controls_tiled(const double* v_grid, int32_t n_v, const double* beta_grid,
                              int32_t n_beta, int64_t n_cand, int32_t n_steps, uint64_t seed,
                              int64_t index_base, int32_t const_prefix, double* tiles,
                              mpc_stream_t stream);
/* Offset (in doubles, from the tiled buffer's base) of candidate c's v at step
 * s; its beta is 512 further. */
static inline int64_t mpc_tiled_index(int64_t c, int32_t s, int32_t n_steps) {
  return (c / MPC_TILE) * 2 * MPC_TILE * (int64_t)n_steps + (int64_t)s * 2 * MPC_TILE +
         c % MPC_TILE;
}


/* ---------------------------------------------------------------------------
 * Device-resident MPC episode: the reference's math_mpc loop
 * (math_model_tree.py:515-635) with its state in HBM, so an MPC step is
 * enqueued with no host synchronisation (graph-capturable):
 *   mpc_episode_expand   grid (:239-256, slow-down :312-316) + sampler +
 *                        rollout + finalize -> local winner
 *   mpc_episode_advance  [multi-GPU: over the all_gather'ed per-rank winners,
 *                        lexicographic (cost, index) selection first]
 *                        finishing logic (:392-414), operator events
 *                        (:564-569), arrival/step-limit restart, one log
 *                        record, then the next step's t += dt (:302), problem
 *                        constants and sampler seed (also done by reset)
 * On one GPU the fused mpc_episode_rollout applies the advance itself
 * (`advance` non-NULL), so a step is two launches (sampler + rollout) — one
 * when the caller supplies the step's candidate controls.
 * The grid ratios are passed precomputed with the reference's expressions.
 * ------------------------------------------------------------------------- */
typedef struct mpc_episode_config {
  double start_x, start_y, start_phi, start_v, start_beta; /* initial_coordinates (:736)   */
  double target_x, target_y;                               /* target_coordinates           */
  double L, delta_t, eps;                                  /* config.py                    */
  double v_max, v_min, delta_v, ratio_v;      /* ratio_v = (v_acc_max*delta_t)/delta_v      */
  double delta_beta, ratio_beta, beta_bound;  /* ratio_beta = degrees(beta_acc_max)*delta_t /
                                                 degrees(delta_beta); beta_bound = beta_max +
                                                 radians(eps_beta)                 (:249-256) */
  double radius_u_turn, turn_distance;                     /* :44; distance 2 (:565-567)   */
  double event_target_x, event_target_y;                   /* new_target(..., 2, 3) (:569) */
  double incumbent0;       /* first optimal_criterion of an episode; 0 = control_criterion of
                              the start pose with the episode's target.  The reference's is
                              computed at import with config.py's target (:676):
                              10000050990.195135                                          */
  int32_t p_turn_right, p_turn_left, p_new_target;         /* 60, 90, 110; <= 0 disables   */
  int32_t slow_new_target, slow_turn;                      /* slow_down(): 10, 20          */
  int32_t max_steps;       /* > 0: restart after this many steps (a safeguard of long benches;
                              the reference has none: 0 = run until on target or stuck)   */
  int32_t enumerate;       /* sampled steps only: 1 = the reference's enumeration — candidate
                              k < |V|*|B| is the constant sequence (V[k / |B|], B[k % |B|])
                              (:311-317), candidates beyond the step's grid are padding with
                              NaN controls (never chosen); 0 = constant prefix + hashed rest */
  int32_t stop_rule;       /* the stuck detector: 0 = math_mpc's (a step that returns the
                              previous pose sets `recursive`, the next step ends the episode,
                              math_model_tree.py:559-563); 1 = run_math_model.py's (the
                              episode's second non-moving step ends it, :266-272)           */
  uint64_t seed;                                           /* candidate sampler seed       */
} mpc_episode_config_t;

/* mpc_episode_log_t.status bits: what math_mpc's loop body (:542-574) did. */
#define MPC_EP_STALE 1    /* no candidate beat the incumbent: the stale optimal_trajectory,
                             result_v, result_beta were applied (:366-429)                 */
#define MPC_EP_STUCK 2    /* the pose equals the previous one: recursive = True (:562-563)  */
#define MPC_EP_BREAK 4    /* recursive was already set: "Recursive error", the episode ended
                             before the events (:559-561); the next step restarts it        */
#define MPC_EP_EVENT 8    /* an operator event fired at this p (:564-569)                   */
#define MPC_EP_ARRIVED 16 /* on target after the step: the episode ended (:542)              */
#define MPC_EP_LIMIT 32   /* max_steps reached: the episode restarts (not in the reference)  */

typedef struct mpc_episode_log {
  int64_t step;          /* global MPC step counter                     */
  int64_t index;         /* chosen candidate (global), -1 if none       */
  int32_t p, episode;    /* iteration number within the episode         */
  int32_t found;         /* a candidate beat the incumbent              */
  int32_t status;        /* MPC_EP_* bits                               */
  double cost, x, y, phi, v, beta;   /* chosen cost and the state moved to */
} mpc_episode_log_t;

size_t mpc_episode_state_bytes(void);
int mpc_episode_reset(const mpc_episode_config_t* cfg, void* state, mpc_stream_t stream);
int mpc_episode_expand(const mpc_episode_config_t* cfg, void* state, double* v_sc,
                       double* beta_sc, int64_t n_cand, int32_t n_steps, int64_t index_base,
                       int32_t integrator, void* ws, size_t ws_bytes, mpc_result_t* out,
                       mpc_stream_t stream);
int mpc_episode_advance(const mpc_episode_config_t* cfg, void* state, const mpc_result_t* results,
                        int32_t n_results, mpc_episode_log_t* log, int32_t log_capacity,
                        mpc_stream_t stream);
/* One launch: streaming rollout + block arg-min, and the last block to finish
 * reduces the block records, re-rolls the winner into `out` and (advance
 * non-NULL, one GPU) applies the episode update.  The step's candidates are
 * v_sc/beta_sc: the sampler's (mpc_episode_sample) or the caller's own.
 * mpc_episode_expand = mpc_episode_sample + this. */
int mpc_episode_rollout(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                        int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                        size_t ws_bytes, mpc_result_t* out, const mpc_episode_config_t* advance,
                        mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream);
/* The launches separately (timing, overlap): grid + sampler | streaming
 * rollout kernel | selection [+ advance]. */
int mpc_episode_sample(const mpc_episode_config_t* cfg, void* state, double* v_sc,
                       double* beta_sc, int64_t n_cand, int32_t n_steps, int64_t index_base,
                       mpc_stream_t stream);
int mpc_episode_partials(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                         int32_t n_steps, int32_t integrator, void* ws, size_t ws_bytes,
                         mpc_stream_t stream);
int mpc_episode_finalize(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                         int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                         size_t ws_bytes, mpc_result_t* out, const mpc_episode_config_t* advance,
                         mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream);
/* mpc_episode_partials + mpc_episode_finalize in one call (the two launches
 * of a step; one host call per step on an eagerly launched episode). */
int mpc_episode_step(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                     int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                     size_t ws_bytes, mpc_result_t* out, const mpc_episode_config_t* advance,
                     mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream);

/* Chained step (integrator MPC_INTEG_RECT | MPC_HEADING_CUMULATIVE, one GPU):
 * ONE launch = the streaming rollout of this step (v_sc / beta_sc, records
 * into ws) + the selection that completes the PREVIOUS step — its records
 * (ws_prev), controls (v_prev / beta_prev; NULL = no previous step) -> winner
 * re-rolled into out_prev, episode update (cfg, log) — run by the launch's
 * first block while the other blocks roll out (they need its published
 * constants only for the final pose transform and the criterion).
 * The last step of a chain is completed by mpc_episode_finalize, which ends
 * the chain.  mode: MPC_CHAIN_FINALIZE.  epoch: nonzero, different from the
 * previous chained launch's.  Aligned path only (n_cand even, 16-B aligned
 * controls): MPC_ERR_UNSUPPORTED otherwise.  ws / ws_prev: two workspaces of
 * mpc_workspace_bytes(n_cand, n_steps) each, alternated.  cfg must be the
 * configuration the state was reset with: the launch picks its wheelbase form
 * (L a power of two or not) from cfg->L, the rollout uses the state's
 * constants; a mismatch sets chain error 2 (mpc_episode_chain_error).
 * hipGraph capture: a captured sequence of chained (or exchange) steps must
 * END with its completing call (mpc_episode_finalize / _exchange_flush), which
 * clears the published constants' epoch tags — a replay repeats the captured
 * epochs, so a sequence left open would let the next replay's launch with the
 * last epoch take the previous replay's constants. */
#define MPC_CHAIN_FINALIZE 1
int mpc_episode_chain_step(const mpc_episode_config_t* cfg, void* state, int32_t mode,
                           uint32_t epoch, const double* v_sc, const double* beta_sc,
                           int64_t n_cand,
                           int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                           const void* ws_prev, size_t ws_bytes, const double* v_prev,
                           const double* beta_prev, mpc_result_t* out_prev,
                           const mpc_result_t* gathered, int32_t n_gathered,
                           mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream);
/* Persistent run (one GPU, integrator MPC_INTEG_RECT | MPC_HEADING_CUMULATIVE,
 * SoA or MPC_LAYOUT_TILED controls under the chained step's rules): n_run
 * COMPLETE MPC steps of the episode — step j over the caller-resident controls
 * v_steps[j] / beta_steps[j] (host arrays of device pointers; tiled: beta =
 * v + 512) — in ONE launch per MPC_RUN_MAX_STEPS steps (math_mpc's loop,
 * math_model_tree.py:515-635): step j+1's candidates stream while step j is
 * selected and applied by the launch's first block (the chained step's
 * completion, mpc_run.h).  Log records, `out` (the last step's winner) and
 * the state are those of n_run chained steps + their finalize, bit for bit.
 * No step may be pending (a chained sequence ends with its finalize first).
 * epoch0: nonzero; the run uses epochs epoch0 .. epoch0 + n_run - 1 (none 0).
 * ws: mpc_episode_run_workspace_bytes(n_cand), zeroed once by the caller (the
 * run leaves it zeroed: graph replays are safe).  A timed-out wait sets chain
 * error 1 (a tile) or 3 (the selector). */
#define MPC_RUN_MAX_STEPS 64
size_t mpc_episode_run_workspace_bytes(int64_t n_cand);
int mpc_episode_run(const mpc_episode_config_t* cfg, void* state, uint32_t epoch0,
                    const double* const* v_steps, const double* const* beta_steps, int32_t n_run,
                    int64_t n_cand, int32_t n_steps, int64_t index_base, int32_t integrator,
                    void* ws, size_t ws_bytes, mpc_result_t* out, mpc_episode_log_t* log,
                    int32_t log_capacity, mpc_stream_t stream);
/* Multi-GPU chained step (same integrator and alignment rules): ONE launch per
 * rank and MPC step, then ONE all_gather of `local` (sizeof(mpc_candidate_t)
 * per rank) by the caller — the all-reduce(min+index) of SURVEY §8e:
 *   block 0: the lexicographic (cost, global index) minimum of the previous
 *            step's gathered per-rank candidates (NULL = no previous step),
 *            re-rolled from its gathered controls into out_prev (the global
 *            winner, on every rank), the episode update, this step's
 *            constants published; then it collects this launch's block
 *            records (16-B granules whose two 8-B halves each carry the
 *            launch's tag: no counter, and no reliance on 16-B single-copy
 *            atomicity) and writes this rank's best candidate (cost, global
 *            index, controls) to `local`;
 *   other blocks: the rollout of this rank's shard (index_base).
 * ws: mpc_workspace_bytes(n_cand, n_steps) (one; consecutive launches are
 * stream-ordered).  The last step is completed by mpc_episode_exchange_flush
 * over its gathered candidates, which ends the chain (and must end a captured
 * sequence, as above).  A collection that timed out sets chain error 3.
 * n_cand < 2^31 (local indices travel in 32 bits of the tagged records). */
int mpc_episode_exchange_step(const mpc_episode_config_t* cfg, void* state, uint32_t epoch,
                              const double* v_sc, const double* beta_sc, int64_t n_cand,
                              int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                              size_t ws_bytes, const mpc_candidate_t* gathered,
                              int32_t n_gathered, mpc_result_t* out_prev, mpc_candidate_t* local,
                              mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream);
/* The exchange step with the collective OFF the launch's critical path: the
 * all_gather of step k runs on another stream beside launch k+1 (it waits on
 * an event recorded after launch k) and is followed there by
 * mpc_episode_exchange_mark(state, epoch of step k); launch k+1 is enqueued
 * with wait_tag = that epoch and needs no stream edge to the collective —
 * only its block 0 waits (bounded; chain error 4 on a timeout) for the mark,
 * then reads the gathered candidates (at most 32 ranks) coherently.  The
 * other blocks roll out step k+1 meanwhile.  The collective's kernel must be
 * able to run beside the launch: on a GPU shared this way, give the launch's
 * stream a CU mask that leaves CUs free for it.  wait_tag 0
 * = mpc_episode_exchange_step (the gathered array already final on the
 * launch's stream). */
int mpc_episode_exchange_step2(const mpc_episode_config_t* cfg, void* state, uint32_t epoch,
                               uint32_t wait_tag, const double* v_sc, const double* beta_sc,
                               int64_t n_cand, int32_t n_steps, int64_t index_base,
                               int32_t integrator, void* ws, size_t ws_bytes,
                               const mpc_candidate_t* gathered, int32_t n_gathered,
                               mpc_result_t* out_prev, mpc_candidate_t* local,
                               mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream);
int mpc_episode_exchange_mark(void* state, uint32_t tag, mpc_stream_t stream);
/* A stream whose kernels leave `reserved_per_xcd` CUs of every XCD (0-8)
 * free for other streams (hipExtStreamCreateWithCUMask): launch the
 * overlapped exchange steps on it, so the collective's kernel (RCCL's needs
 * ~280 registers per wave, which never fit beside a chained launch that
 * fills a CU) always finds CUs.  The mask is a property of the stream a
 * kernel or a replayed hipGraph is launched on.  MPC_ERR_UNSUPPORTED on any
 * device but a 256-CU gfx950 (the CU -> XCD layout the mask assumes was
 * measured there).  Release with mpc_stream_destroy after synchronising. */
int mpc_stream_create_cu_reserved(int32_t reserved_per_xcd, mpc_stream_t* stream);
/* A stream whose kernels run on the `part`-th of `parts` disjoint CU sets
 * (CU j of every XCD belongs to part j % parts): ranks that REHEARSE a
 * multi-GPU run on fewer GPUs launch on disjoint sets, so one rank's chained
 * launch (whose tiles wait for block 0, which waits for the peers) can never
 * occupy the CUs a peer's block 0 needs.  Same device restriction and
 * release as above. */
int mpc_stream_create_cu_share(int32_t part, int32_t parts, mpc_stream_t* stream);
int mpc_stream_destroy(mpc_stream_t stream);
int mpc_episode_exchange_flush(const mpc_episode_config_t* cfg, void* state, int32_t integrator,
                               const mpc_candidate_t* gathered, int32_t n_gathered,
                               mpc_result_t* out, mpc_episode_log_t* log, int32_t log_capacity,
                               mpc_stream_t stream);
/* Multi-GPU chained step WITHOUT a collective (SURVEY §8e over xGMI): the
 * per-rank candidates travel by peer stores from the launches themselves, and
 * the exchange of step k runs inside launch k+1 beside its rollout.  Every
 * rank owns a mailbox (mpc_mailbox_alloc: mpc_mailbox_bytes(world) bytes of
 * its HBM, zeroed; uncached = 1 makes every access go to HBM, which is what
 * peer stores over xGMI need to be seen) whose header holds the world
 * mailboxes as mapped in this process (mpc_mailbox_set_peers, once, before
 * the first step; peers[rank] = this mailbox): another process's via
 * mpc_ipc_handle (on its rank) + mpc_ipc_open (here), another GPU of this
 * process directly after mpc_peer_enable.  Per MPC step each rank launches
 *   mpc_episode_p2p_step(epoch, prev_epoch = the previous step's epoch, 0 on
 *   the first step of a chain) — the structure of mpc_episode_chain_step
 *   (ws / ws_prev alternated, the previous step's controls v_prev / beta_prev)
 *   whose block 0 reduces the previous launch's block records into this
 *   rank's candidate, stores it into slot prev_epoch & 1 of every rank's
 *   mailbox (then the tags), waits (bounded, 2 s; chain error 5) for the
 *   world candidates in its own mailbox, selects the (cost, global index)
 *   minimum, re-rolls it into out_prev (the global winner, on every rank),
 *   updates the episode and publishes this step's constants; the tile blocks
 *   meanwhile roll out this rank's shard (index_base).
 * Consecutive epochs must differ in parity; the mailbox slot is chosen on the
 * device by the episode's count of P2P completions; every rank runs the same
 * sequence of epochs.  The chain ends with
 * mpc_episode_p2p_flush (the last step's controls and workspace).  No host
 * step and no collective between launches: plain kernels on one stream,
 * graph-capturable (end a captured sequence with the flush, as above).
 * world <= 32. */
#define MPC_IPC_HANDLE_BYTES 64
size_t mpc_mailbox_bytes(int32_t world);
int mpc_mailbox_alloc(int32_t world, int32_t uncached, void** mailbox);
int mpc_mailbox_free(void* mailbox);
int mpc_mailbox_set_peers(void* mailbox, int32_t rank, int32_t world, const void* const* peers);
/* Self-test of the mailboxes (every rank, after every rank's set_peers, e.g.
 * behind a barrier): each rank stores `tag` into every rank's ping word and
 * waits (~0.1 s at most) for all of its own; *ok (device int32) = 1 if all
 * arrived.  A host that gets 0 on any rank uses the all_gather exchange. */
int mpc_mailbox_ping(void* mailbox, uint32_t tag, int32_t* ok, mpc_stream_t stream);
/* Zero this rank's candidate slots (not the header) on `stream`: with the
 * episode's reset, so that a step replayed with an epoch of an earlier run
 * (a HIP graph captured before the reset) never reads a stale granule whose
 * tag matches.  Call it while no peer stores into this mailbox. */
int mpc_mailbox_clear(void* mailbox, int32_t world, mpc_stream_t stream);
int mpc_ipc_handle(void* dev_ptr, void* handle /* MPC_IPC_HANDLE_BYTES */);
int mpc_ipc_open(const void* handle, void** dev_ptr);
int mpc_ipc_close(void* dev_ptr);
int mpc_peer_enable(int32_t peer_device);
int mpc_episode_p2p_step(const mpc_episode_config_t* cfg, void* state, uint32_t epoch,
                         uint32_t prev_epoch, const double* v_sc, const double* beta_sc,
                         int64_t n_cand, int32_t n_steps, int64_t index_base, int32_t integrator,
                         void* ws, const void* ws_prev, size_t ws_bytes, const double* v_prev,
                         const double* beta_prev, void* mailbox, int32_t world,
                         mpc_result_t* out_prev, mpc_episode_log_t* log, int32_t log_capacity,
                         mpc_stream_t stream);
int mpc_episode_p2p_flush(const mpc_episode_config_t* cfg, void* state, uint32_t last_epoch,
                          const double* v_last, const double* beta_last, int64_t n_cand,
                          int32_t n_steps, int64_t index_base, int32_t integrator,
                          const void* ws_last, size_t ws_bytes, void* mailbox, int32_t world,
                          mpc_result_t* out, mpc_episode_log_t* log, int32_t log_capacity,
                          mpc_stream_t stream);

/* The exchange's collective for a non-Python host: an RCCL
 * communicator per GPU — one process driving all local GPUs (a clique,
 * mpc_comm_init_all) or one rank per process (mpc_comm_unique_id on rank 0,
 * shared by the caller, then mpc_comm_init_rank on every rank) — and the
 * per-step all_gather of the ranks' mpc_candidate_t (device pointers; the
 * gathered array has one record per rank, in rank order).  RCCL is loaded at
 * run time (librccl.so.1); MPC_ERR_UNSUPPORTED if it cannot be.
 * mpc_exchange_allgather_group issues n communicators' all_gathers inside one
 * RCCL group (the single-process clique: one thread, one stream per GPU). */
typedef struct mpc_comm* mpc_comm_t;
int mpc_comm_unique_id(void* id /* 128 bytes */);
int mpc_comm_init_rank(const void* id, int32_t n_ranks, int32_t rank, mpc_comm_t* comm);
int mpc_comm_init_all(int32_t n_devices, const int32_t* devices, mpc_comm_t* comms);
int mpc_comm_destroy(mpc_comm_t comm);
int mpc_exchange_allgather(mpc_comm_t comm, const mpc_candidate_t* local,
                           mpc_candidate_t* gathered, mpc_stream_t stream);
int mpc_exchange_allgather_group(int32_t n, const mpc_comm_t* comms,
                                 const mpc_candidate_t* const* local,
                                 mpc_candidate_t* const* gathered, const mpc_stream_t* streams);

/* Generated controls (one GPU): one MPC step of the device-resident episode
 * whose candidates are never materialised — the same candidates, bit for bit,
 * as mpc_episode_sample followed by mpc_episode_step (advance = cfg) on the
 * sampler's arrays: every block builds the step's grid (math_model_tree.py
 * :239-256, slow-down :312-316) in LDS and draws each candidate-step's entry
 * with the sampler's hash (constant prefix included), rolls it out, and the
 * selection re-rolls the winner and advances the episode.  n_cand even;
 * ws: mpc_episode_generate_workspace_bytes(n_cand, n_steps).  The grid (at
 * most 64 x 64 entries) is staged in LDS. */
size_t mpc_episode_generate_workspace_bytes(int64_t n_cand, int32_t n_steps);
int mpc_episode_generate_step(const mpc_episode_config_t* cfg, void* state, int64_t n_cand,
                              int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                              size_t ws_bytes, mpc_result_t* out, mpc_episode_log_t* log,
                              int32_t log_capacity, mpc_stream_t stream);
/* Nonzero if a chained step went wrong: 1 = a chained step's wait for the
 * published constants timed out (the launch then ran on stale constants);
 * 2 = cfg's wheelbase form disagreed with the state's; 3 = an exchange step's
 * collection of its block records timed out (`local` then holds none); 4 = an
 * overlapped exchange step's wait for the gathered candidates' mark timed out
 * (the step was not completed: the episode kept its pose); 5 = a P2P exchange
 * step's wait for the ranks' candidates in its mailbox timed out (a peer did
 * not run the same step; the step was not completed, and the later steps of
 * the episode fail fast instead of waiting again); 6 = a one-GPU chained
 * step's early publication of the next constants (formed from the new pose
 * before the rest of the update, in a step without event or restart)
 * differed from the update's own (a self-check: never expected).
 * The waits are bounded on the GPU's wall clock: 0.2 s for a one-GPU chained
 * launch's tiles; 2 s for block 0's wait for peers or a collective (4, 5); 3 s
 * for the tiles of an exchange / P2P launch, so a late peer is never scored as
 * error 1.  A multi-rank caller reduces the code over its ranks (a rank that
 * timed out posts no candidate, so its peers' steps are suspect too).
 * Reads the device state (syncs). */
int mpc_episode_chain_error(const void* state, int32_t* error, mpc_stream_t stream);

/* ---------------------------------------------------------------------------
 * Batched device-resident episodes: run_math_model.py's loop
 * (:231-280) over R robots — each its own episode (start, target, rules in
 * its mpc_episode_config_t) whose MPC step is math_model_tree.py's tree
 * expansion: the grid around the robot's (v, beta) (:239-256, slow-down
 * :312-316), the reference's enumeration of its |V|*|B| constant sequences
 * (:308-350, at most 64 x 64), the n_steps-layer rollout, the strict-< first
 * minimum against the robot's incumbent (:351), the winner's layer states, the
 * update of mpc_episode_advance (finishing logic, cfg.stop_rule's stuck
 * detector, events when enabled, arrival, cfg.max_steps) — without restart: an
 * ended episode stops its robot.  ONE launch runs up to max_calls MPC steps of
 * every robot (one block per robot, no host round trip, no lockstep);
 * repeated launches continue the episodes.  cfg.enumerate is implied.
 *   mpc_episodes_reset   copies the R configurations (host array, validated)
 *                        into the state and starts every episode (a robot that
 *                        starts on its target is stopped at once)
 *   mpc_episodes_run     log: [R][log_capacity] rings of mpc_episode_log_t
 *                        (slot = step % capacity, nullable); progress: device
 *                        array [R], written at the end of the launch
 * ------------------------------------------------------------------------- */
typedef struct mpc_episodes_progress {
  int32_t calls;         /* MPC steps run so far                                     */
  int32_t stop;          /* 0 = running; else the MPC_EP_* bits of the step that ended
                            the episode (MPC_EP_ARRIVED with calls 0: started on target) */
  int64_t candidates;    /* candidates rolled out so far (sum of the steps' |V|*|B|)   */
} mpc_episodes_progress_t;
size_t mpc_episodes_state_bytes(int32_t n_robots);
int mpc_episodes_reset(const mpc_episode_config_t* cfgs, int32_t n_robots, void* state,
                       mpc_stream_t stream);
int mpc_episodes_run(void* state, int32_t n_robots, int32_t n_steps, int32_t integrator,
                     int32_t max_calls, mpc_episode_log_t* log, int32_t log_capacity,
                     mpc_episodes_progress_t* progress, mpc_stream_t stream);

/* ---------------------------------------------------------------------------
 * Full-tree MPC of run_math_model.py / math_model.py.
 * predictive_control (run_math_model.py:133-228) fills S1^3 leaves, S1 =
 * |V|*|B|: leaf j = k0*S1^2 + k1*S1 + k2 applies u_k0, u_k1, u_k2 in turn
 * (u_k = (V[k / |B|], B[k % |B|]), the :158-160 loop order) and is scored with
 * the heading-term criterion (:82-86)
 *   10000*dist_target + 10*(arctan(x_t/y_t) - phi)^2 + 100*dist_line^2,
 * strict < against an incumbent that the reference never resets within an
 * episode (:193-196).  Leaves are generated from j: nothing per leaf in HBM.
 * The caller passes arctan(x_t / y_t) as its numpy evaluates it (:83).
 * ------------------------------------------------------------------------- */
typedef struct mpc_fulltree_problem {
  double x, y, phi;           /* initial_coordinates (:139)                     */
  double x_t, y_t, x_0, y_0;  /* module globals read by the criterion (:56-86)  */
  double atan_target;         /* arctan(x_t / y_t) (:83)                        */
  double L, t_a, t_b;         /* quad window [t, t + delta_t] after t += dt      */
} mpc_fulltree_problem_t;

typedef struct mpc_fulltree_result {
  double cost;                /* criterion of the best leaf                     */
  int64_t leaf;               /* j of the first strict minimum, -1 if none      */
  int32_t found;              /* cost < incumbent                               */
  int32_t s1;                 /* |V| * |B|                                      */
  int64_t k[3];               /* control index per layer                        */
  double v[3], beta[3];       /* the controls                                   */
  double traj[3][3];          /* layer states (x, y, phi) of the best leaf      */
} mpc_fulltree_result_t;

size_t mpc_fulltree_workspace_bytes(int32_t n_v, int32_t n_beta);
/* v_grid / beta_grid: device arrays; out: device pointer.  shard / n_shards:
 * this call evaluates the shard-th of n_shards contiguous parts of the leaf
 * set (leaf indices stay global); the winner over all shards is the
 * lexicographic (cost, leaf) minimum of the shards' results (multi-GPU:
 * one all_gather of the results per MPC step). */
int mpc_fulltree_argmin(const mpc_fulltree_problem_t* p, const double* v_grid, int32_t n_v,
                        const double* beta_grid, int32_t n_beta, double incumbent,
                        int32_t integrator, int32_t shard, int32_t n_shards, void* ws,
                        size_t ws_bytes, mpc_fulltree_result_t* out, mpc_stream_t stream);

/* R robots' full trees in one launch sequence (the run_math_model.py:231-280
 * episodes side by side, one robot per episode, stepping in lockstep).
 * problems / incumbents / out: device arrays [n_problems]; the problems' L,
 * t_a, t_b are ignored: every robot uses (L, t_a, t_b) given here (lockstep
 * robots share the MPC step's quad window).  Problem constants are derived
 * on the device (squares as x*x). */
size_t mpc_fulltree_batched_workspace_bytes(int32_t n_problems, int32_t n_v, int32_t n_beta);
int mpc_fulltree_argmin_batched(const mpc_fulltree_problem_t* problems,
                                const double* incumbents, int32_t n_problems, double L,
                                double t_a, double t_b, const double* v_grid, int32_t n_v,
                                const double* beta_grid, int32_t n_beta, int32_t integrator,
                                void* ws, size_t ws_bytes, mpc_fulltree_result_t* out,
                                mpc_stream_t stream);

/* ---------------------------------------------------------------------------
 * Full-tree episodes, device-resident: run_math_model.py's
 * episode loop (:231-280) with its OWN full-tree MPC step (:133-228, the tree
 * of mpc_fulltree_argmin) for R robots, one robot per episode.  ONE call
 * enqueues up to max_calls MPC steps of every robot (per-robot state in HBM,
 * no host round trip): per MPC step three launches over the robots still
 * running — compaction and the step's control table, every live robot's
 * leaves spread over the whole GPU, one update per live robot (live robots
 * have run the same number of calls: one quad window, one table).  Per call:
 * the stop rules before it (on target :261, the robot's max_calls), t +=
 * delta_t (:156), the S1^3
 * leaves scored with the heading-term criterion, strict < against the robot's
 * never-reset optimal_criterion (:193-196), the winner's first layer as the
 * returned state (or the stale one when no leaf wins), the two-non-move stop
 * (:266-272).  Repeated launches continue the episodes.
 *   mpc_fulltree_episodes_reset  copies the R configurations (host array; the
 *                                caller evaluates the script's expressions for
 *                                atan_target and incumbent0) into the state
 *   mpc_fulltree_episodes_run    v_grid / beta_grid: device arrays, S1 <= 512;
 *                                log: [R][log_capacity] rings (slot = step %
 *                                capacity; cost = optimal_criterion after the
 *                                call, index = the winning leaf or -1); progress:
 *                                {calls, stop, leaves scored} per robot
 * A robot whose first call finds no winning leaf stops with MPC_EP_NO_TRAJ (the
 * script raises TypeError there: optimal_trajectory is still [0]).
 * ------------------------------------------------------------------------- */
#define MPC_EP_NO_TRAJ 64
typedef struct mpc_fulltree_episode_config {
  double x_0, y_0, phi_0;     /* start (:235-237)                                    */
  double x_t, y_t;            /* target (:238-239)                                   */
  double atan_target;         /* numpy arctan(x_t / y_t) (:83)                       */
  double incumbent0;          /* control_criterion([x_0, y_0, phi_0]) (:252)        */
  int32_t max_calls;          /* MPC calls after which the episode stops; 0 = none  */
  int32_t reserved_;
} mpc_fulltree_episode_config_t;
size_t mpc_fulltree_episodes_state_bytes(int32_t n_robots);
int mpc_fulltree_episodes_reset(const mpc_fulltree_episode_config_t* cfgs, int32_t n_robots,
                                void* state, mpc_stream_t stream);
int mpc_fulltree_episodes_run(void* state, int32_t n_robots, const double* v_grid, int32_t n_v,
                              const double* beta_grid, int32_t n_beta, double L, double delta_t,
                              double eps, int32_t integrator, int32_t max_calls,
                              mpc_episode_log_t* log, int32_t log_capacity,
                              mpc_episodes_progress_t* progress, mpc_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DIPLOMJOURNEY_AMD_MPC_ROLLOUT_H */
