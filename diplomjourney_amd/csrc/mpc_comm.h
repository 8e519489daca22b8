// mpc_comm.h — the multi-GPU exchange's collective for a non-Python host
// (the RCCL clique and the per-step all-reduce(min+index) entry).
// RCCL is resolved at run time (dlopen "librccl.so.1"): a Python process that
// already loaded torch's RCCL reuses it (same soname), a C/C++ host loads
// ROCm's, and the library itself keeps no link-time RCCL dependency.  The
// handful of entry points used are declared here with RCCL's ABI.
#pragma once

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/mpc_rollout.h"

namespace mpc {
namespace rccl {

typedef struct ncclComm* Comm;
typedef struct {
  char internal[128];
} UniqueId;
constexpr int kSuccess = 0;
constexpr int kUint8 = 1;   // ncclUint8

struct Api {
  int (*get_unique_id)(UniqueId*) = nullptr;
  int (*comm_init_rank)(Comm*, int, UniqueId, int) = nullptr;
  int (*comm_init_all)(Comm*, int, const int*) = nullptr;
  int (*comm_destroy)(Comm) = nullptr;
  int (*all_gather)(const void*, void*, size_t, int, Comm, hipStream_t) = nullptr;
  int (*group_start)() = nullptr;
  int (*group_end)() = nullptr;
  bool ok = false;
};

inline const Api& api() {
  static Api a = [] {
    Api r;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    r.get_unique_id = reinterpret_cast<int (*)(UniqueId*)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank =
        reinterpret_cast<int (*)(Comm*, int, UniqueId, int)>(dlsym(h, "ncclCommInitRank"));
    r.comm_init_all = reinterpret_cast<int (*)(Comm*, int, const int*)>(dlsym(h, "ncclCommInitAll"));
    r.comm_destroy = reinterpret_cast<int (*)(Comm)>(dlsym(h, "ncclCommDestroy"));
    r.all_gather = reinterpret_cast<int (*)(const void*, void*, size_t, int, Comm, hipStream_t)>(
        dlsym(h, "ncclAllGather"));
    r.group_start = reinterpret_cast<int (*)()>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<int (*)()>(dlsym(h, "ncclGroupEnd"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_init_all && r.comm_destroy &&
           r.all_gather && r.group_start && r.group_end;
    return r;
  }();
  return a;
}

}  // namespace rccl
}  // namespace mpc
