// Image-parallel group of include/mathocr.h (BASELINE config 3):
// one process per GPU, each rank encodes and decodes its own shard of the global batch
// with no collective on the data path, then the decoded token streams are all-gathered
// over RCCL (xGMI) into every rank's device memory.
//
// RCCL is opened at run time (dlopen of librccl.so.1, RTLD_LOCAL) so that libmathocr.so
// loads without it and its symbols never interpose with the RCCL a host framework may
// have loaded; only rccl.h's types are used at compile time.  The gather runs on the
// group's own HIP stream and returns when the result is in place.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/mathocr.h"
#include "kernels.h"

static_assert(NCCL_UNIQUE_ID_BYTES == MOCR_GROUP_ID_BYTES, "RCCL unique id size");

namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

template <typename F>
void bind(void* h, F& fn, const char* name) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  if (!fn) throw std::runtime_error(std::string("librccl: missing symbol ") + name);
}

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    x.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!x.h) x.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!x.h) throw std::runtime_error(std::string("cannot load librccl.so.1: ") + dlerror());
    bind(x.h, x.get_unique_id, "ncclGetUniqueId");
    bind(x.h, x.comm_init_rank, "ncclCommInitRank");
    bind(x.h, x.comm_destroy, "ncclCommDestroy");
    bind(x.h, x.comm_count, "ncclCommCount");
    bind(x.h, x.all_gather, "ncclAllGather");
    bind(x.h, x.error_string, "ncclGetErrorString");
    return x;
  }();
  return r;
}

void check(ncclResult_t rc, const char* what) {
  if (rc != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + rccl().error_string(rc));
}

thread_local std::string g_group_error;

int group_fail(const std::exception& ex) {
  g_group_error = ex.what();
  if (auto* he = dynamic_cast<const mocr::HipError*>(&ex)) return -1000 - (int)he->code;
  return -1;
}

}  // namespace

struct mocr_group {
  ncclComm_t comm = nullptr;
  int world = 0, rank = 0, device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ready = nullptr;  // the caller's stream state, waited on by the group stream
  int32_t* shapes = nullptr;   // device [world][2]: every rank's (rows, width), checked before a gather
  int32_t* shapes_host = nullptr;
};

extern "C" {

const char* mocr_group_last_error(void) { return g_group_error.c_str(); }

int mocr_group_unique_id(uint8_t* id_out) {
  try {
    if (!id_out) throw std::runtime_error("null id_out");
    ncclUniqueId id;
    check(rccl().get_unique_id(&id), "ncclGetUniqueId");
    std::memcpy(id_out, id.internal, MOCR_GROUP_ID_BYTES);
    return 0;
  } catch (const std::exception& ex) {
    return group_fail(ex);
  }
}

int mocr_group_create(const uint8_t* id, int world, int rank, int hip_device, mocr_group** out) {
  mocr_group* g = nullptr;
  try {
    if (!id || !out) throw std::runtime_error("null argument");
    if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("rank / world out of range");
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, MOCR_GROUP_ID_BYTES);
    g = new mocr_group();
    g->world = world;
    g->rank = rank;
    g->device = hip_device;
    MOCR_HIP_CHECK(hipSetDevice(hip_device));
    MOCR_HIP_CHECK(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    MOCR_HIP_CHECK(hipEventCreateWithFlags(&g->ready, hipEventDisableTiming));
    MOCR_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&g->shapes), (size_t)world * 2 * sizeof(int32_t)));
    MOCR_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&g->shapes_host), (size_t)world * 2 * sizeof(int32_t),
                                 hipHostMallocDefault));
    check(rccl().comm_init_rank(&g->comm, world, uid, rank), "ncclCommInitRank");
    *out = g;
    return 0;
  } catch (const std::exception& ex) {
    if (g) {
      if (g->stream) (void)hipStreamDestroy(g->stream);
      if (g->ready) (void)hipEventDestroy(g->ready);
      if (g->shapes) (void)hipFree(g->shapes);
      if (g->shapes_host) (void)hipHostFree(g->shapes_host);
      delete g;
    }
    if (out) *out = nullptr;
    return group_fail(ex);
  }
}

int mocr_group_destroy(mocr_group* g) {
  if (!g) return 0;
  (void)hipSetDevice(g->device);
  if (g->comm) (void)rccl().comm_destroy(g->comm);
  if (g->stream) (void)hipStreamDestroy(g->stream);
  if (g->ready) (void)hipEventDestroy(g->ready);
  if (g->shapes) (void)hipFree(g->shapes);
  if (g->shapes_host) (void)hipHostFree(g->shapes_host);
  delete g;
  return 0;
}

int mocr_group_size(const mocr_group* g, int* ranks_out) {
  try {
    if (!g || !ranks_out) throw std::runtime_error("null argument");
    check(rccl().comm_count(g->comm, ranks_out), "ncclCommCount");
    return 0;
  } catch (const std::exception& ex) {
    return group_fail(ex);
  }
}

int mocr_group_gather_ids(mocr_group* g, const int32_t* ids_dev, int rows, int width, int32_t* ids_all_dev,
                          void* producer_stream) {
  try {
    if (!g || !ids_dev || !ids_all_dev) throw std::runtime_error("null argument");
    if (rows < 0 || width < 1) throw std::runtime_error("rows / width out of range");
    MOCR_HIP_CHECK(hipSetDevice(g->device));
    // the ids (and the reuse of ids_all_dev) are ordered behind the producer's stream
    MOCR_HIP_CHECK(hipEventRecord(g->ready, static_cast<hipStream_t>(producer_stream)));
    MOCR_HIP_CHECK(hipStreamWaitEvent(g->stream, g->ready, 0));
    // every rank must pass the same shape: all-gather the (rows, width) pairs first, so an
    // uneven shard fails here on every rank instead of hanging or corrupting the gather
    const int32_t mine[2] = {rows, width};
    MOCR_HIP_CHECK(hipMemcpyAsync(g->shapes + 2 * g->rank, mine, sizeof(mine), hipMemcpyHostToDevice, g->stream));
    check(rccl().all_gather(g->shapes + 2 * g->rank, g->shapes, 2, ncclInt32, g->comm, g->stream), "ncclAllGather");
    MOCR_HIP_CHECK(hipMemcpyAsync(g->shapes_host, g->shapes, (size_t)g->world * 2 * sizeof(int32_t),
                                  hipMemcpyDeviceToHost, g->stream));
    MOCR_HIP_CHECK(hipStreamSynchronize(g->stream));
    for (int r = 0; r < g->world; ++r)
      if (g->shapes_host[2 * r] != rows || g->shapes_host[2 * r + 1] != width)
        throw std::runtime_error("mocr_group_gather_ids: rank " + std::to_string(r) + " passes [" +
                                 std::to_string(g->shapes_host[2 * r]) + ", " + std::to_string(g->shapes_host[2 * r + 1]) +
                                 "], rank " + std::to_string(g->rank) + " [" + std::to_string(rows) + ", " +
                                 std::to_string(width) + "]: shards must be equal (pad them to the same rows)");
    check(rccl().all_gather(ids_dev, ids_all_dev, (size_t)rows * width, ncclInt32, g->comm, g->stream),
          "ncclAllGather");
    MOCR_HIP_CHECK(hipStreamSynchronize(g->stream));
    return 0;
  } catch (const std::exception& ex) {
    return group_fail(ex);
  }
}

}  // extern "C"
