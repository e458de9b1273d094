// rccl_comm.cpp — RCCL collectives over the GPUs one aggregator process drives (include/fedagg.h,
// "shard group" section).
//
// FedScale's aggregator is ONE process: every upload lands in it (aggregator.py:919-963) and egress is
// served from its gRPC servicer threads (aggregator.py:871-917).  To spread a round over the node's GPUs
// behind that unmodified event loop, the library drives N devices from the one process and the
// cross-device steps are RCCL collectives over xGMI issued for all N devices at once
// (ncclCommInitAll + ncclGroupStart/End, one stream per device).  No rendezvous, no second process.
//
// RCCL is resolved at run time (dlopen): the copy torch already loaded is reused when present, so one
// RCCL lives in the process; the library itself has no link-time dependency on it and loads on hosts
// without RCCL (fa_rccl_available() then returns 0 and fa_rccl_init fails with FA_E_HIP).
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <new>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../include/fedagg.h"
#include "fa_device.h"

namespace {

struct RcclApi {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGetVersion) version = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommCuDevice) cu_device = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
  decltype(&ncclGetUniqueId) unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  bool ok = false;
};

RcclApi g_api;
std::once_flag g_api_once;

void load_api() {
  // the RCCL torch loaded (soname librccl.so.1) first; else the ROCm install's
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return;
#define FA_SYM(field, name) g_api.field = reinterpret_cast<decltype(g_api.field)>(dlsym(h, name))
  FA_SYM(init_all, "ncclCommInitAll");
  FA_SYM(destroy, "ncclCommDestroy");
  FA_SYM(group_start, "ncclGroupStart");
  FA_SYM(group_end, "ncclGroupEnd");
  FA_SYM(all_gather, "ncclAllGather");
  FA_SYM(all_reduce, "ncclAllReduce");
  FA_SYM(gather, "ncclGather");
  FA_SYM(broadcast, "ncclBroadcast");
  FA_SYM(error_string, "ncclGetErrorString");
  FA_SYM(version, "ncclGetVersion");
  FA_SYM(count, "ncclCommCount");
  FA_SYM(cu_device, "ncclCommCuDevice");
  FA_SYM(user_rank, "ncclCommUserRank");
  FA_SYM(unique_id, "ncclGetUniqueId");
  FA_SYM(init_rank, "ncclCommInitRank");
#undef FA_SYM
  g_api.ok = g_api.init_all && g_api.destroy && g_api.group_start && g_api.group_end && g_api.all_gather &&
             g_api.all_reduce && g_api.gather && g_api.broadcast && g_api.error_string && g_api.count &&
             g_api.cu_device && g_api.user_rank && g_api.unique_id && g_api.init_rank;
}

const RcclApi* api() {
  std::call_once(g_api_once, load_api);
  return g_api.ok ? &g_api : nullptr;
}

struct Comm {
  int n = 0;                       // communicators this handle holds (the devices this process drives)
  std::vector<ncclComm_t> comms;
  std::vector<int> devs;  // device of comms[i]
};

int err(int code, const char* what, ncclResult_t r) {
  char buf[256];
  const RcclApi* a = api();
  snprintf(buf, sizeof(buf), "%s: %s", what, a ? a->error_string(r) : "RCCL unavailable");
  return fa_internal_set_error(code, buf);
}

int dtype_of(int32_t dt, ncclDataType_t* out, size_t* elem) {
  switch (dt) {
    case FA_DT_F32: *out = ncclFloat32; *elem = 4; return FA_OK;
    case FA_DT_F64: *out = ncclFloat64; *elem = 8; return FA_OK;
    case FA_DT_I64: *out = ncclInt64; *elem = 8; return FA_OK;
    default: return fa_internal_set_error(FA_E_ARG, "fa_rccl: unknown dtype");
  }
}

int check(void* comm, int64_t count, const char* what, Comm** c) {
  if (!api()) return fa_internal_set_error(FA_E_HIP, "fa_rccl: RCCL could not be loaded");
  if (!comm || count < 0) return fa_internal_set_error(FA_E_ARG, what);
  *c = static_cast<Comm*>(comm);
  return FA_OK;
}

// streams[i] must be a stream of device devs[i]: HIP would resolve a NULL stream against whatever device is
// current when RCCL enqueues, so a group over several devices takes explicit per-device streams
int check_streams(const Comm* c, void* const* streams, const char* what) {
  char buf[256];
  for (int i = 0; i < c->n; ++i) {
    hipStream_t st = (hipStream_t)streams[i];
    if (st == nullptr || st == hipStreamPerThread) {
      if (c->n == 1) continue;
      snprintf(buf, sizeof(buf), "%s: streams[%d] is NULL; a group over %d devices needs a stream per device", what,
               i, c->n);
      return fa_internal_set_error(FA_E_ARG, buf);
    }
    int d = -1;
    if (hipStreamGetDevice(st, &d) != hipSuccess) {
      (void)hipGetLastError();
      snprintf(buf, sizeof(buf), "%s: streams[%d] is not a valid stream", what, i);
      return fa_internal_set_error(FA_E_ARG, buf);
    }
    if (d != c->devs[i]) {
      snprintf(buf, sizeof(buf), "%s: streams[%d] belongs to device %d, the communicator's rank %d is device %d",
               what, i, d, i, c->devs[i]);
      return fa_internal_set_error(FA_E_ARG, buf);
    }
  }
  return FA_OK;
}

// the buffer of rank i (bytes of it) must be device memory of the communicator's device i (fa_device.h): a
// buffer on another GPU would be read over xGMI by the wrong rank's kernels, pageable memory would fault the GPU
int check_buf(const Comm* c, const char* what, void* const* streams, int i, const char* name, const void* p,
              uint64_t bytes) {
  if (!p) {
    char buf[160];
    snprintf(buf, sizeof(buf), "%s: %s[%d] is NULL", what, name, i);
    return fa_internal_set_error(FA_E_ARG, buf);
  }
  DevScope scope(what, streams[i], p);
  if (scope.rc() != FA_OK) return scope.rc();
  if (scope.device() != c->devs[i]) {
    char buf[200];
    snprintf(buf, sizeof(buf), "%s: %s[%d] is memory of device %d, the communicator's rank %d is device %d", what,
             name, i, scope.device(), i, c->devs[i]);
    return fa_internal_set_error(FA_E_ARG, buf);
  }
  char nm[48];
  snprintf(nm, sizeof(nm), "%s[%d]", name, i);
  return scope.operand(nm, p, bytes);
}

// one grouped launch: op(i) issues device i's part of the collective
template <class F>
int grouped(const Comm* c, const char* what, F op) {
  const RcclApi* a = api();
  ncclResult_t r = a->group_start();
  if (r != ncclSuccess) return err(FA_E_HIP, what, r);
  ncclResult_t first = ncclSuccess;
  for (int i = 0; i < c->n; ++i) {
    r = op(i);
    if (r != ncclSuccess && first == ncclSuccess) first = r;
  }
  r = a->group_end();  // always close the group, even after a failed enqueue
  if (first != ncclSuccess) return err(FA_E_HIP, what, first);
  if (r != ncclSuccess) return err(FA_E_HIP, what, r);
  return FA_OK;
}

}  // namespace

extern "C" int fa_rccl_available(void) { return api() ? 1 : 0; }

extern "C" int fa_rccl_init(int32_t ndev, const int32_t* devs, void** comm_out) {
  if (ndev < 1 || !devs || !comm_out) return fa_internal_set_error(FA_E_ARG, "fa_rccl_init: bad arguments");
  for (int i = 0; i < ndev; ++i)
    for (int j = 0; j < i; ++j)
      if (devs[i] == devs[j])
        return fa_internal_set_error(FA_E_ARG, "fa_rccl_init: a device appears twice (one rank per GPU)");
  const RcclApi* a = api();
  if (!a) return fa_internal_set_error(FA_E_HIP, "fa_rccl_init: RCCL could not be loaded");
  Comm* c = new (std::nothrow) Comm();
  if (!c) return fa_internal_set_error(FA_E_HIP, "fa_rccl_init: out of memory");
  c->n = ndev;
  c->comms.resize(ndev);
  c->devs.assign(devs, devs + ndev);
  std::vector<int> d(devs, devs + ndev);
  ncclResult_t r = a->init_all(c->comms.data(), ndev, d.data());
  if (r != ncclSuccess) {
    delete c;
    return err(FA_E_HIP, "fa_rccl_init: ncclCommInitAll", r);
  }
  *comm_out = c;
  return FA_OK;
}

// One rank of a communicator that spans processes (one process per GPU): the bench's SPMD ranks open one over
// their own GPU to record what RCCL itself sees (fa_rccl_comm_info), next to torch.distributed's view.
extern "C" int fa_rccl_unique_id(void* id_out) {
  if (!id_out) return fa_internal_set_error(FA_E_ARG, "fa_rccl_unique_id: NULL");
  const RcclApi* a = api();
  if (!a) return fa_internal_set_error(FA_E_HIP, "fa_rccl_unique_id: RCCL could not be loaded");
  ncclUniqueId id;
  ncclResult_t r = a->unique_id(&id);
  if (r != ncclSuccess) return err(FA_E_HIP, "fa_rccl_unique_id: ncclGetUniqueId", r);
  memcpy(id_out, &id, sizeof(id));
  return FA_OK;
}

extern "C" int fa_rccl_init_rank(int32_t nranks, const void* id, int32_t rank, int32_t device, void** comm_out) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !id || !comm_out || device < 0)
    return fa_internal_set_error(FA_E_ARG, "fa_rccl_init_rank: bad arguments");
  const RcclApi* a = api();
  if (!a) return fa_internal_set_error(FA_E_HIP, "fa_rccl_init_rank: RCCL could not be loaded");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    return fa_internal_set_error(FA_E_HIP, "fa_rccl_init_rank: cannot select the device");
  }
  Comm* c = new (std::nothrow) Comm();
  if (!c) {
    (void)hipSetDevice(prev);
    return fa_internal_set_error(FA_E_HIP, "fa_rccl_init_rank: out of memory");
  }
  c->n = 1;
  c->comms.resize(1);
  c->devs.assign(1, device);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclResult_t r = a->init_rank(c->comms.data(), nranks, uid, rank);  // collective over the nranks processes
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) {
    delete c;
    return err(FA_E_HIP, "fa_rccl_init_rank: ncclCommInitRank", r);
  }
  *comm_out = c;
  return FA_OK;
}

// What RCCL reports for a handle: its rank count (ncclCommCount, the same on every communicator of the handle or
// FA_E_HIP), and for each of the handle's communicators i its rank (ncclCommUserRank) and device
// (ncclCommCuDevice).  `ranks` / `devs` hold one entry per communicator of the handle (fa_rccl_init: ndev;
// fa_rccl_init_rank: 1); either may be NULL.
extern "C" int fa_rccl_comm_info(void* comm, int32_t* count, int32_t* ranks, int32_t* devs) {
  Comm* c;
  int e = check(comm, 0, "fa_rccl_comm_info: bad arguments", &c);
  if (e) return e;
  if (!count) return fa_internal_set_error(FA_E_ARG, "fa_rccl_comm_info: NULL count");
  const RcclApi* a = api();
  int n0 = -1;
  for (int i = 0; i < c->n; ++i) {
    int n = -1, rk = -1, d = -1;
    ncclResult_t r = a->count(c->comms[i], &n);
    if (r == ncclSuccess) r = a->user_rank(c->comms[i], &rk);
    if (r == ncclSuccess) r = a->cu_device(c->comms[i], &d);
    if (r != ncclSuccess) return err(FA_E_HIP, "fa_rccl_comm_info", r);
    if (i > 0 && n != n0) return fa_internal_set_error(FA_E_HIP, "fa_rccl_comm_info: the communicators disagree "
                                                                  "on the rank count");
    n0 = n;
    if (ranks) ranks[i] = rk;
    if (devs) devs[i] = d;
  }
  *count = n0;
  return FA_OK;
}

extern "C" int fa_rccl_destroy(void* comm) {
  if (!comm) return FA_OK;
  Comm* c = static_cast<Comm*>(comm);
  const RcclApi* a = api();
  int rc = FA_OK;
  if (a)
    for (ncclComm_t x : c->comms) {
      ncclResult_t r = a->destroy(x);
      if (r != ncclSuccess && rc == FA_OK) rc = err(FA_E_HIP, "fa_rccl_destroy", r);
    }
  delete c;
  return rc;
}

extern "C" int fa_rccl_all_gather(void* comm, const void* const* send, void* const* recv, int64_t count,
                                  int32_t dtype, void* const* streams) {
  Comm* c;
  int e = check(comm, count, "fa_rccl_all_gather: bad arguments", &c);
  if (e) return e;
  ncclDataType_t dt;
  size_t sz;
  if ((e = dtype_of(dtype, &dt, &sz))) return e;
  if (!send || !recv || !streams) return fa_internal_set_error(FA_E_ARG, "fa_rccl_all_gather: NULL table");
  if ((e = check_streams(c, streams, "fa_rccl_all_gather"))) return e;
  for (int i = 0; i < c->n && count > 0; ++i)
    if ((e = check_buf(c, "fa_rccl_all_gather", streams, i, "send", send[i], (uint64_t)count * sz)) ||
        (e = check_buf(c, "fa_rccl_all_gather", streams, i, "recv", recv[i], (uint64_t)count * sz * c->n)))
      return e;
  const RcclApi* a = api();
  return grouped(c, "fa_rccl_all_gather", [&](int i) {
    return a->all_gather(send[i], recv[i], (size_t)count, dt, c->comms[i], (hipStream_t)streams[i]);
  });
}

extern "C" int fa_rccl_all_reduce(void* comm, const void* const* send, void* const* recv, int64_t count,
                                  int32_t dtype, void* const* streams) {
  Comm* c;
  int e = check(comm, count, "fa_rccl_all_reduce: bad arguments", &c);
  if (e) return e;
  ncclDataType_t dt;
  size_t sz;
  if ((e = dtype_of(dtype, &dt, &sz))) return e;
  if (!send || !recv || !streams) return fa_internal_set_error(FA_E_ARG, "fa_rccl_all_reduce: NULL table");
  if ((e = check_streams(c, streams, "fa_rccl_all_reduce"))) return e;
  for (int i = 0; i < c->n && count > 0; ++i)
    if ((e = check_buf(c, "fa_rccl_all_reduce", streams, i, "send", send[i], (uint64_t)count * sz)) ||
        (e = check_buf(c, "fa_rccl_all_reduce", streams, i, "recv", recv[i], (uint64_t)count * sz)))
      return e;
  const RcclApi* a = api();
  return grouped(c, "fa_rccl_all_reduce", [&](int i) {
    return a->all_reduce(send[i], recv[i], (size_t)count, dt, ncclSum, c->comms[i], (hipStream_t)streams[i]);
  });
}

extern "C" int fa_rccl_gather(void* comm, const void* const* send, void* recv_root, int64_t count, int32_t dtype,
                              int32_t root, void* const* streams) {
  Comm* c;
  int e = check(comm, count, "fa_rccl_gather: bad arguments", &c);
  if (e) return e;
  ncclDataType_t dt;
  size_t sz;
  if ((e = dtype_of(dtype, &dt, &sz))) return e;
  if (!send || !recv_root || !streams || root < 0 || root >= c->n)
    return fa_internal_set_error(FA_E_ARG, "fa_rccl_gather: bad root or NULL table");
  if ((e = check_streams(c, streams, "fa_rccl_gather"))) return e;
  for (int i = 0; i < c->n && count > 0; ++i)
    if ((e = check_buf(c, "fa_rccl_gather", streams, i, "send", send[i], (uint64_t)count * sz)))
      return e;
  if (count > 0 && (e = check_buf(c, "fa_rccl_gather", streams, root, "recv_root", recv_root,
                                  (uint64_t)count * sz * c->n)))
    return e;
  const RcclApi* a = api();
  return grouped(c, "fa_rccl_gather", [&](int i) {
    return a->gather(send[i], i == root ? recv_root : nullptr, (size_t)count, dt, root, c->comms[i],
                     (hipStream_t)streams[i]);
  });
}

extern "C" int fa_rccl_broadcast(void* comm, void* const* bufs, int64_t count, int32_t dtype, int32_t root,
                                 void* const* streams) {
  Comm* c;
  int e = check(comm, count, "fa_rccl_broadcast: bad arguments", &c);
  if (e) return e;
  ncclDataType_t dt;
  size_t sz;
  if ((e = dtype_of(dtype, &dt, &sz))) return e;
  if (!bufs || !streams || root < 0 || root >= c->n)
    return fa_internal_set_error(FA_E_ARG, "fa_rccl_broadcast: bad root or NULL table");
  if ((e = check_streams(c, streams, "fa_rccl_broadcast"))) return e;
  for (int i = 0; i < c->n && count > 0; ++i)
    if ((e = check_buf(c, "fa_rccl_broadcast", streams, i, "bufs", bufs[i], (uint64_t)count * sz))) return e;
  const RcclApi* a = api();
  return grouped(c, "fa_rccl_broadcast", [&](int i) {
    return a->broadcast(bufs[i], bufs[i], (size_t)count, dt, root, c->comms[i], (hipStream_t)streams[i]);
  });
}
