// Gradient all-reduce straight from the C ABI over RCCL (xGMI on MI355X).
//
// The reference averages gradients through DistributedDataParallel's bucketed NCCL
// all-reduce (train.py:947-951 wraps the model; data/utils.py:40-44 reduce_tensor for
// the logged loss).  SURVEY §8b names the op `allreduce_bucket` over an opaque
// `ds2_comm_t` created from an ncclUniqueId that torch.distributed (or a file) carries
// to every rank.  This file is that: one communicator per rank, an in-place SUM of one
// contiguous fp32 bucket of the flat gradient buffer enqueued on the caller's stream
// (the caller scales by 1/world after the last bucket, as GradAllReducer does, so the
// result is DDP's average bit for bit for power-of-two worlds).
//
// RCCL is resolved at run time (dlopen of librccl.so.1): a process that imported torch
// already holds torch's RCCL under that soname and shares it; nothing else in the
// library depends on RCCL being present.
#include <dlfcn.h>
#include <string.h>

#include <rccl/rccl.h>

#include "common.h"

struct ds2_comm {
  ncclComm_t comm;
  int nranks;
  int rank;
};

namespace {

struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const RcclApi& rccl() {
  static const RcclApi api = [] {
    RcclApi a;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) return a;
    a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    a.all_reduce = reinterpret_cast<decltype(a.all_reduce)>(dlsym(h, "ncclAllReduce"));
    a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(h, "ncclGetErrorString"));
    a.ok = a.get_unique_id && a.comm_init_rank && a.all_reduce && a.comm_destroy && a.error_string;
    return a;
  }();
  return api;
}

ds2_status_t rccl_status(const char* where, ncclResult_t r) {
  if (r == ncclSuccess) return DS2_OK;
  ds2::set_last_error_text(where, rccl().error_string(r));
  return DS2_RCCL_ERROR;
}

ds2_status_t rccl_missing(const char* where) {
  ds2::set_last_error_text(where, "librccl.so.1 could not be loaded");
  return DS2_RCCL_ERROR;
}

}  // namespace

extern "C" {

size_t ds2_comm_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

ds2_status_t ds2_comm_get_unique_id(void* id_out) {
  if (id_out == nullptr) return DS2_INVALID_VALUE;
  if (!rccl().ok) return rccl_missing("ds2_comm_get_unique_id");
  ncclUniqueId id;
  const ds2_status_t s = rccl_status("ds2_comm_get_unique_id", rccl().get_unique_id(&id));
  if (s == DS2_OK) memcpy(id_out, &id, sizeof(id));
  return s;
}

ds2_status_t ds2_comm_init(ds2_comm_t* comm, const void* id, int nranks, int rank, int device) {
  if (comm == nullptr || id == nullptr || nranks < 1 || rank < 0 || rank >= nranks || device < 0)
    return DS2_INVALID_VALUE;
  *comm = nullptr;
  if (!rccl().ok) return rccl_missing("ds2_comm_init");
  const hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    ds2::set_last_error("ds2_comm_init", e);
    return DS2_HIP_ERROR;
  }
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const ds2_status_t s =
      rccl_status("ds2_comm_init", rccl().comm_init_rank(&c, nranks, uid, rank));
  if (s != DS2_OK) return s;
  *comm = new ds2_comm{c, nranks, rank};
  return DS2_OK;
}

ds2_status_t ds2_allreduce_bucket(ds2_comm_t comm, float* bucket, int64_t count,
                                  ds2_stream_t stream) {
  if (comm == nullptr || count < 0 || (count > 0 && bucket == nullptr)) return DS2_INVALID_VALUE;
  if (count == 0) return DS2_OK;
  return rccl_status("ds2_allreduce_bucket",
                     rccl().all_reduce(bucket, bucket, static_cast<size_t>(count), ncclFloat32,
                                       ncclSum, comm->comm, static_cast<hipStream_t>(stream)));
}

ds2_status_t ds2_comm_destroy(ds2_comm_t comm) {
  if (comm == nullptr) return DS2_OK;
  const ds2_status_t s = rccl_status("ds2_comm_destroy", rccl().comm_destroy(comm->comm));
  delete comm;
  return s;
}

}  // extern "C"
