// exchange_episode.cpp — a C++ host (no Python) driving the sharded
// device-resident MPC episode through the C ABI only: ONE process, n_dev GPUs
// (an RCCL clique, mpc_comm_init_all), per MPC step one
// mpc_episode_exchange_step per GPU and one grouped RCCL all_gather of the
// ranks' candidates (mpc_exchange_allgather_group); the chain is ended by
// mpc_episode_exchange_flush.  Used by tests/test_gpu_parity.py::
// test_c_host_exchange_episode (built by __graft_entry__.build()).
//
//   exchange_episode IN.bin OUT.bin
// IN.bin: int32 n_dev, n_steps, steps, n_v, n_b, pad; int64 n_total;
//         uint64 seed0; mpc_episode_config_t; double V[n_v]; double B[n_b]
// OUT.bin: per device, `steps` mpc_episode_log_t records (ring order by step),
//          then per device its final winner (mpc_result_t).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/mpc_rollout.h"

#define CK(x)                                                                  \
  do {                                                                         \
    int s_ = (x);                                                              \
    if (s_ != 0) {                                                             \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, s_,     \
              s_ < 0 ? mpc_strerror(s_) : "hip");                              \
      return 1;                                                                \
    }                                                                          \
  } while (0)

struct Rank {
  hipStream_t st;
  void *state, *ws;
  size_t ws_bytes;
  double *v, *b, *vg, *bg;   // [4 batches][n_steps][n_local] controls; grids
  mpc_candidate_t *cand, *gathered;
  mpc_result_t* winner;
  mpc_episode_log_t* log;
  int64_t lo, n_local;
};

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s IN.bin OUT.bin\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t hdr[6];
  int64_t n_total;
  uint64_t seed0;
  mpc_episode_config_t cfg;
  if (fread(hdr, sizeof(hdr), 1, f) != 1 || fread(&n_total, 8, 1, f) != 1 ||
      fread(&seed0, 8, 1, f) != 1 || fread(&cfg, sizeof(cfg), 1, f) != 1)
    return 2;
  const int n_dev = hdr[0], n_steps = hdr[1], steps = hdr[2], n_v = hdr[3], n_b = hdr[4];
  std::vector<double> V(n_v), B(n_b);
  if (fread(V.data(), 8, n_v, f) != static_cast<size_t>(n_v) ||
      fread(B.data(), 8, n_b, f) != static_cast<size_t>(n_b))
    return 2;
  fclose(f);
  const int kBatches = 4;
  const int log_cap = steps + 4;
  std::vector<Rank> R(n_dev);
  std::vector<int32_t> devs(n_dev);
  for (int d = 0; d < n_dev; ++d) devs[d] = d;
  std::vector<mpc_comm_t> comms(n_dev);
  CK(mpc_comm_init_all(n_dev, devs.data(), comms.data()));
  const int integ = MPC_INTEG_RECT | MPC_HEADING_CUMULATIVE;
  for (int d = 0; d < n_dev; ++d) {
    Rank& r = R[d];
    CK(hipSetDevice(d));
    CK(hipStreamCreateWithFlags(&r.st, hipStreamNonBlocking));
    const int64_t base = n_total / n_dev, rem = n_total % n_dev;   // contiguous shards
    r.lo = d * base + (d < rem ? d : rem);
    r.n_local = base + (d < rem ? 1 : 0);
    CK(hipMalloc(&r.state, mpc_episode_state_bytes()));
    CK(hipMemset(r.state, 0, mpc_episode_state_bytes()));
    r.ws_bytes = mpc_workspace_bytes(r.n_local, n_steps);
    CK(hipMalloc(&r.ws, r.ws_bytes));
    const size_t per = static_cast<size_t>(n_steps) * r.n_local;
    CK(hipMalloc(&r.v, kBatches * per * 8));
    CK(hipMalloc(&r.b, kBatches * per * 8));
    CK(hipMalloc(&r.vg, n_v * 8));
    CK(hipMalloc(&r.bg, n_b * 8));
    CK(hipMemcpy(r.vg, V.data(), n_v * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(r.bg, B.data(), n_b * 8, hipMemcpyHostToDevice));
    for (int k = 0; k < kBatches; ++k)   // this rank's shard of batch k (global indices)
      CK(mpc_sample_controls(r.vg, n_v, r.bg, n_b, r.n_local, n_steps, seed0 + k, r.lo, 1,
                             r.v + k * per, r.b + k * per, r.n_local, r.st));
    CK(hipMalloc(&r.cand, sizeof(mpc_candidate_t)));
    CK(hipMalloc(&r.gathered, n_dev * sizeof(mpc_candidate_t)));
    CK(hipMalloc(&r.winner, sizeof(mpc_result_t)));
    CK(hipMemset(r.winner, 0, sizeof(mpc_result_t)));
    CK(hipMalloc(&r.log, log_cap * sizeof(mpc_episode_log_t)));
    CK(hipMemset(r.log, 0, log_cap * sizeof(mpc_episode_log_t)));
    CK(mpc_episode_reset(&cfg, r.state, r.st));
  }
  std::vector<const mpc_candidate_t*> locals(n_dev);
  std::vector<mpc_candidate_t*> gathers(n_dev);
  std::vector<mpc_stream_t> streams(n_dev);
  for (int d = 0; d < n_dev; ++d) {
    locals[d] = R[d].cand;
    gathers[d] = R[d].gathered;
    streams[d] = reinterpret_cast<mpc_stream_t>(R[d].st);
  }
  for (int s = 0; s < steps; ++s) {
    for (int d = 0; d < n_dev; ++d) {
      Rank& r = R[d];
      CK(hipSetDevice(d));
      const size_t per = static_cast<size_t>(n_steps) * r.n_local;
      const int k = s % kBatches;
      CK(mpc_episode_exchange_step(&cfg, r.state, static_cast<uint32_t>(s + 1), r.v + k * per,
                                   r.b + k * per, r.n_local, n_steps, r.lo, integ, r.ws,
                                   r.ws_bytes, s ? r.gathered : nullptr, n_dev, r.winner, r.cand,
                                   r.log, log_cap, streams[d]));
    }
    CK(mpc_exchange_allgather_group(n_dev, comms.data(), locals.data(), gathers.data(),
                                    streams.data()));
  }
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 2;
  std::vector<mpc_episode_log_t> host(log_cap);
  for (int d = 0; d < n_dev; ++d) {
    Rank& r = R[d];
    CK(hipSetDevice(d));
    CK(mpc_episode_exchange_flush(&cfg, r.state, integ, r.gathered, n_dev, r.winner, r.log,
                                  log_cap, streams[d]));
    int32_t err = 0;
    CK(mpc_episode_chain_error(r.state, &err, streams[d]));
    if (err) {
      fprintf(stderr, "device %d: chain error %d\n", d, err);
      return 1;
    }
    CK(hipMemcpy(host.data(), r.log, log_cap * sizeof(mpc_episode_log_t), hipMemcpyDeviceToHost));
    for (int s = 0; s < steps; ++s) fwrite(&host[s % log_cap], sizeof(mpc_episode_log_t), 1, o);
  }
  for (int d = 0; d < n_dev; ++d) {
    mpc_result_t w;
    CK(hipSetDevice(d));
    CK(hipMemcpy(&w, R[d].winner, sizeof(w), hipMemcpyDeviceToHost));
    fwrite(&w, sizeof(w), 1, o);
    CK(mpc_comm_destroy(comms[d]));
  }
  fclose(o);
  printf("ok %d devices, %d steps\n", n_dev, steps);
  return 0;
}
