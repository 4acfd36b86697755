// Data-parallel communicator: one RCCL communicator per process over the ranks of
// the job, behind the C ABI of include/manette_hip.h (mt_comm_*). The reference has no
// collective of its own — its only shard unit is the contiguous env split of runners.py:17-18 —
// so the one exchange of a data-parallel update is this build's: ONE in-place sum all-reduce of
// the flat fp32 gradient per update (2.7 MB NIPS .. 6.8 MB NATURE), enqueued on the learner's
// stream between the backward and mt_clip_rmsprop (which folds the 1/world scale in), plus the
// start-of-run broadcast of rank 0's parameters and RMSProp slots. Both are plain stream-ordered
// RCCL calls, so they can be captured into the update's hipGraph (mt_graph_*).
#include <rccl/rccl.h>

#include <algorithm>

#include "common.h"

static_assert(NCCL_UNIQUE_ID_BYTES == MT_COMM_UID_BYTES, "RCCL unique id size");

struct mt_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
  // loopback (mt_comm_init_loopback, tests): no RCCL; the "sum" of `replicas` identical replicas
  float replicas = 0.f;
  uint64_t delay_ticks = 0;
};

using namespace mt;

#define MT_RCCL(call)                                                                              \
  do {                                                                                             \
    ncclResult_t r_ = (call);                                                                      \
    if (r_ != ncclSuccess) {                                                                       \
      set_error("%s failed: %s (%s:%d)", #call, ncclGetErrorString(r_), __FILE__, __LINE__);       \
      return MT_ERR_HIP;                                                                           \
    }                                                                                              \
  } while (0)

extern "C" int mt_comm_unique_id(char *uid) {
  MT_CHECK_ARG(uid, "null argument");
  ncclUniqueId id;
  MT_RCCL(ncclGetUniqueId(&id));
  std::memcpy(uid, id.internal, MT_COMM_UID_BYTES);
  return MT_OK;
}

extern "C" int mt_comm_init(const char *uid, int rank, int world, int device, mt_comm **out) {
  MT_CHECK_ARG(uid && out, "null argument");
  MT_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "rank %d out of [0, %d)", rank, world);
  MT_HIP(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(id.internal, uid, MT_COMM_UID_BYTES);
  ncclComm_t c;
  MT_RCCL(ncclCommInitRank(&c, world, id, rank));
  mt_comm *m = new mt_comm();
  m->comm = c;
  m->rank = rank;
  m->world = world;
  m->device = device;
  *out = m;
  return MT_OK;
}

extern "C" int mt_comm_init_loopback(int replicas, int delay_us, mt_comm **out) {
  MT_CHECK_ARG(out, "null argument");
  MT_CHECK_ARG(replicas >= 1 && delay_us >= 0 && delay_us <= 100000, "replicas %d / delay %d us", replicas, delay_us);
  mt_comm *m = new mt_comm();
  m->replicas = (float)replicas;
  m->delay_ticks = (uint64_t)delay_us * 100;  // s_memrealtime: 100 MHz
  *out = m;
  return MT_OK;
}

extern "C" void mt_comm_destroy(mt_comm *comm) {
  if (!comm) return;
  if (comm->comm) (void)ncclCommDestroy(comm->comm);
  delete comm;
}

// loopback all-reduce: scale by the replica count at once (a sum that started before its producer
// finished would be overwritten), then hold the stream for delay_ticks (a consumer that does not
// wait for the sum would run first)
__global__ __launch_bounds__(256) void loopback_sum_kernel(float *buf, size_t n, float replicas) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) buf[i] *= replicas;
}
__global__ void loopback_delay_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" int mt_comm_info(const mt_comm *comm, int *rank, int *world) {
  MT_CHECK_ARG(comm, "null argument");
  if (rank) *rank = comm->rank;
  if (world) *world = comm->world;
  return MT_OK;
}

extern "C" int mt_allreduce(mt_comm *comm, float *buf, size_t n, mt_stream_t stream) {
  MT_CHECK_ARG(comm && (buf || n == 0), "null argument");
  if (n == 0) return MT_OK;
  if (!comm->comm) {  // loopback
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(loopback_sum_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, buf, n, comm->replicas);
    MT_HIP(hipGetLastError());
    if (comm->delay_ticks) {
      hipLaunchKernelGGL(loopback_delay_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, comm->delay_ticks);
      MT_HIP(hipGetLastError());
    }
    return MT_OK;
  }
  MT_RCCL(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, comm->comm, (hipStream_t)stream));
  return MT_OK;
}

extern "C" int mt_broadcast(mt_comm *comm, void *buf, size_t bytes, int root, mt_stream_t stream) {
  MT_CHECK_ARG(comm && (buf || bytes == 0), "null argument");
  MT_CHECK_ARG(root >= 0 && root < comm->world, "root %d out of [0, %d)", root, comm->world);
  if (bytes == 0 || !comm->comm) return MT_OK;  // (loopback: the replicas are identical)
  MT_RCCL(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm->comm, (hipStream_t)stream));
  return MT_OK;
}
