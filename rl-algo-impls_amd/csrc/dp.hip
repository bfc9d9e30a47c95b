// Data-parallel runtime: RCCL communicator + the per-minibatch
//   grads kernel -> ncclAllReduce (xGMI) -> clip + Adam
// loop of one PPO epoch, driven natively so the host enqueues each optimizer step in a few
// microseconds (the Python-level loop costs ~3x that per step, which at 2,048 steps per epoch
// would leave the GPU idle between the collectives).
//
// RCCL is resolved at run time from the librccl.so.1 the process already mapped (PyTorch-ROCm
// links it; same SONAME), so this library has no link-time RCCL dependency and there is one
// RCCL in the process.  Replaces the reference's single-process optimizer loop
// (rl_algo_impls/ppo/ppo.py:290-411) for the multi-GPU case of SURVEY.md 8(e).
#include <dlfcn.h>

#include <cstring>

#include "common.h"

namespace {

struct RcclUid {
  char internal[RAI_DP_UID_BYTES];
};
typedef int (*GetUniqueIdFn)(RcclUid*);
typedef int (*CommInitRankFn)(void**, int, RcclUid, int);
typedef int (*CommDestroyFn)(void*);
typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, void*, hipStream_t);
typedef const char* (*ErrStrFn)(int);

constexpr int NCCL_FLOAT32 = 7;  // ncclFloat32
constexpr int NCCL_SUM = 0;      // ncclSum

struct Rccl {
  GetUniqueIdFn get_uid = nullptr;
  CommInitRankFn init = nullptr;
  CommDestroyFn destroy = nullptr;
  AllReduceFn allreduce = nullptr;
  ErrStrFn errstr = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return x;
    x.get_uid = reinterpret_cast<GetUniqueIdFn>(dlsym(h, "ncclGetUniqueId"));
    x.init = reinterpret_cast<CommInitRankFn>(dlsym(h, "ncclCommInitRank"));
    x.destroy = reinterpret_cast<CommDestroyFn>(dlsym(h, "ncclCommDestroy"));
    x.allreduce = reinterpret_cast<AllReduceFn>(dlsym(h, "ncclAllReduce"));
    x.errstr = reinterpret_cast<ErrStrFn>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_uid && x.init && x.destroy && x.allreduce;
    return x;
  }();
  return r;
}

// RCCL errors are reported as RAI_E_DP_BASE - ncclResult_t
int rccl_rc(int r) { return r == 0 ? RAI_OK : RAI_E_DP_BASE - r; }

}  // namespace

// mlp_ppo.hip (C++ linkage): multi-CU grads kernel that first applies the previous all-reduced step
int rai_mlp_ppo_dp_step(float* params, float* exp_avg, float* exp_avg_sq, const float* grad_in, int32_t P_total,
                        const float* obs, const int64_t* actions, const float* old_logp, const float* old_values,
                        const float* advantages, const float* returns, int64_t n_rows, int32_t batch_size,
                        int32_t mb, int32_t mb_count, const float* moments, int32_t world, int32_t in_dim,
                        int32_t hidden, int32_t n_actions, int32_t activation, const rai_ppo_hparams* hp,
                        const rai_optim_hparams* ohp, rai_train_state* state, float* grad_out, float* stats,
                        int32_t max_stats, float* norms, int32_t max_norms, int32_t sync_base, void* workspace,
                        int64_t workspace_bytes, void* stream);

extern "C" int rai_dp_available(void) { return rccl().ok ? 1 : 0; }

extern "C" int rai_dp_unique_id(void* out, int32_t out_bytes) {
  if (!out) return RAI_E_NULLPTR;
  if (out_bytes < RAI_DP_UID_BYTES) return RAI_E_SHAPE;
  if (!rccl().ok) return RAI_E_UNSUPPORTED;
  RcclUid uid;
  const int r = rccl().get_uid(&uid);
  if (r != 0) return rccl_rc(r);
  memcpy(out, uid.internal, RAI_DP_UID_BYTES);
  return RAI_OK;
}

extern "C" int rai_dp_comm_init(void** comm_out, const void* uid_bytes, int32_t world, int32_t rank) {
  if (!comm_out || !uid_bytes) return RAI_E_NULLPTR;
  if (world < 1 || rank < 0 || rank >= world) return RAI_E_SHAPE;
  if (!rccl().ok) return RAI_E_UNSUPPORTED;
  RcclUid uid;
  memcpy(uid.internal, uid_bytes, RAI_DP_UID_BYTES);
  return rccl_rc(rccl().init(comm_out, world, uid, rank));
}

extern "C" int rai_dp_comm_destroy(void* comm) {
  if (!comm) return RAI_E_NULLPTR;
  if (!rccl().ok) return RAI_E_UNSUPPORTED;
  return rccl_rc(rccl().destroy(comm));
}

extern "C" int rai_dp_allreduce_sum_f32(void* comm, float* buf, int64_t n, void* stream) {
  if (!comm || !buf) return RAI_E_NULLPTR;
  if (n < 0) return RAI_E_SHAPE;
  if (!rccl().ok) return RAI_E_UNSUPPORTED;
  return rccl_rc(rccl().allreduce(buf, buf, (size_t)n, NCCL_FLOAT32, NCCL_SUM, comm, rai_stream(stream)));
}

extern "C" int rai_mlp_ppo_epoch_dp(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t P,
                                    const float* obs, const int64_t* actions, const float* old_logp,
                                    const float* old_values, const float* advantages, const float* returns,
                                    int64_t n_rows, int32_t batch_size, const float* moments, int32_t world,
                                    int32_t in_dim, int32_t hidden, int32_t n_actions, int32_t activation,
                                    const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
                                    rai_train_state* state, float* stats, int32_t max_stats, float* norms,
                                    int32_t max_norms, void* comm, float* grads_alt, void* workspace,
                                    int64_t workspace_bytes, void* optim_workspace, int64_t optim_workspace_bytes,
                                    void* stream) {
  if (!comm || !grads || !moments) return RAI_E_NULLPTR;
  if (batch_size < 1 || n_rows < 1 || P < 1) return RAI_E_SHAPE;
  const int64_t nmb = (n_rows + batch_size - 1) / batch_size;
  if (grads_alt && P <= INT32_MAX) {
    // Two launches per optimizer step: the multi-CU kernel applies step k-1's all-reduced gradient
    // (clip + Adam on every CU's weight copy) and computes step k's partial gradient; RCCL sums it.
    // The gradient buffers alternate so step k's kernel never overwrites what it is applying.
    float* buf[2] = {grads, grads_alt};
    int rc = RAI_OK;
    for (int64_t mb = 0; mb <= nmb; ++mb) {
      const float* gin = mb == 0 ? nullptr : buf[(mb - 1) & 1];
      float* gout = buf[mb & 1];
      rc = rai_mlp_ppo_dp_step(params, exp_avg, exp_avg_sq, gin, (int32_t)P, obs, actions, old_logp, old_values,
                               advantages, returns, n_rows, batch_size, (int32_t)(mb < nmb ? mb : 0),
                               mb < nmb ? 1 : 0, moments, world, in_dim, hidden, n_actions, activation, hp, ohp,
                               state, gout, stats, max_stats, norms, max_norms, (int32_t)mb, workspace,
                               workspace_bytes, stream);
      if (rc == RAI_E_UNSUPPORTED && mb == 0) break;  // not the multi-CU layout: three-call loop below
      if (rc != RAI_OK) return rc;
      if (mb < nmb) {
        rc = rai_dp_allreduce_sum_f32(comm, gout, P, stream);
        if (rc != RAI_OK) return rc;
      }
    }
    if (rc == RAI_OK) return RAI_OK;
  }
  for (int64_t mb = 0; mb < nmb; ++mb) {
    int rc = rai_mlp_ppo_grads(params, obs, actions, old_logp, old_values, advantages, returns, n_rows, batch_size,
                               (int32_t)mb, 1, moments, world, in_dim, hidden, n_actions, activation, hp, ohp, state,
                               grads, stats, max_stats, workspace, workspace_bytes, stream);
    if (rc != RAI_OK) return rc;
    rc = rai_dp_allreduce_sum_f32(comm, grads, P, stream);
    if (rc != RAI_OK) return rc;
    rc = rai_clip_optim_step(params, grads, exp_avg, exp_avg_sq, P, ohp, state, norms, max_norms, optim_workspace,
                             optim_workspace_bytes, stream);
    if (rc != RAI_OK) return rc;
  }
  return RAI_OK;
}

// ---- cross-GPU exchange regions (in-kernel all-reduce over xGMI peer memory) -------------------
// Uncached device memory (every access goes to HBM, so a peer's stores are visible to this
// device's loads without cache maintenance), shared with the other ranks' processes by IPC.
extern "C" int rai_xdp_alloc(int64_t bytes, void** region_out) {
  if (!region_out) return RAI_E_NULLPTR;
  if (bytes <= 0) return RAI_E_SHAPE;
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, (size_t)bytes);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return (int)e;
  }
  *region_out = p;
  return RAI_OK;
}

extern "C" int rai_xdp_free(void* region) {
  if (!region) return RAI_E_NULLPTR;
  return (int)hipFree(region);
}

extern "C" int rai_xdp_handle(void* region, void* handle_out, int32_t out_bytes) {
  if (!region || !handle_out) return RAI_E_NULLPTR;
  if (out_bytes < (int32_t)sizeof(hipIpcMemHandle_t)) return RAI_E_SHAPE;
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, region);
  if (e != hipSuccess) return (int)e;
  memcpy(handle_out, &h, sizeof(h));
  return RAI_OK;
}

extern "C" int rai_xdp_open(const void* handle, void** peer_region_out) {
  if (!handle || !peer_region_out) return RAI_E_NULLPTR;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(peer_region_out, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int rai_xdp_close(void* peer_region) {
  if (!peer_region) return RAI_E_NULLPTR;
  return (int)hipIpcCloseMemHandle(peer_region);
}

extern "C" int rai_xdp_handle_bytes(void) { return (int)sizeof(hipIpcMemHandle_t); }
