// lego_comm.hip — the stream-per-GPU hand-off collective behind
// the C-ABI: every rank's batch packet (lego_handoff_pack: pose records plus
// the published corner / surf / outlier "last" clouds of
// featureAssociation.cpp:1790-1815) gathered to the rank that runs the serial
// mapping consumer, over RCCL (xGMI between the GPUs of a node).
//
// One collective per batch: ncclGather of the 8-byte packet sizes, then one
// group of ncclSend (every other rank) / ncclRecv (root, one per peer), so
// each peer's packet travels on its own link.  Root's own packet is a
// device-to-device copy.  The received packets are copied to pinned host
// memory for the host-side consumers (lego_handoff_unpack -> lego_mo_process),
// or, with LEGO_COMM_DEVICE_RESULT, stay in HBM and nothing waits for the
// transfer (the next call does: the sender's packet buffer is reused then).
//
// Failure policy: a rank whose pack fails sends an empty packet, so the
// others never wait for it; an RCCL or device error once the communicator is
// in use closes any open group and aborts the communicator (ncclCommAbort),
// and the communicator is dead from then on.  Only root sizes buffers after
// the size exchange; it aborts if that fails.  Every wait on the
// communicator's stream is bounded (lego_comm_set_timeout, default 60 s): a
// peer that never joins a collective makes the call abort the communicator
// and return LEGO_E_DEVICE naming the wait, instead of blocking the rank.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "lego_loam.h"

void lego_set_error(const char* fmt, ...);  // lego_api.hip
// lego_api.hip: the send of lego_handoff_pack's buffer in flight on stream s
// (an event the next pack into that buffer waits for)
extern "C" int lego_handoff_fence(lego_ctx* ctx, hipStream_t s);

struct lego_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
  hipStream_t s = nullptr;
  uint64_t* dSize = nullptr;   // [1] this rank's packet size
  uint64_t* dSizes = nullptr;  // [nranks] gathered on root
  uint8_t* dRecv = nullptr;    // root: every packet, back to back
  size_t recvCap = 0;
  uint8_t* hRecv = nullptr;    // pinned copy of dRecv
  size_t hCap = 0;
  std::vector<uint64_t> sizes, offs;
  bool haveResult = false, haveHost = false;
  bool dead = false;
  int timeoutMs = 60000;  // bound of every wait on s (lego_comm_set_timeout)
  ~lego_comm() {
    if (device >= 0) (void)hipSetDevice(device);
    if (s) (void)hipStreamSynchronize(s);
    if (nc) (void)ncclCommDestroy(nc);
    if (dSize) (void)hipFree(dSize);
    if (dSizes) (void)hipFree(dSizes);
    if (dRecv) (void)hipFree(dRecv);
    if (hRecv) (void)hipHostFree(hRecv);
    if (s) (void)hipStreamDestroy(s);
  }
};

#define COMM_HIP(call)                                                      \
  do {                                                                      \
    hipError_t e_ = (call);                                                 \
    if (e_ != hipSuccess) {                                                 \
      lego_set_error("%s: %s", #call, hipGetErrorString(e_));               \
      return LEGO_E_DEVICE;                                                 \
    }                                                                       \
  } while (0)
#define COMM_NCCL(call)                                                     \
  do {                                                                      \
    ncclResult_t r_ = (call);                                               \
    if (r_ != ncclSuccess) {                                                \
      lego_set_error("%s: %s", #call, ncclGetErrorString(r_));              \
      return LEGO_E_DEVICE;                                                 \
    }                                                                       \
  } while (0)

extern "C" {

int lego_comm_unique_id(uint8_t id[128]) {
  if (!id) return LEGO_E_ARG;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId u;
  COMM_NCCL(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return LEGO_OK;
}

int lego_comm_create(const uint8_t id[128], int32_t nranks, int32_t rank, int32_t device, lego_comm** out) {
  if (!id || !out || nranks <= 0 || rank < 0 || rank >= nranks || device < 0) return LEGO_E_ARG;
  *out = nullptr;
  lego_comm* c = new lego_comm;
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  auto fail = [&](int st) {
    delete c;
    return st;
  };
  if (hipSetDevice(device) != hipSuccess) {
    lego_set_error("lego_comm_create: no HIP device %d", device);
    return fail(LEGO_E_DEVICE);
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->nc, nranks, u, rank);
  if (r != ncclSuccess) {
    c->nc = nullptr;
    lego_set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
    return fail(LEGO_E_DEVICE);
  }
  if (hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->dSize, sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&c->dSizes, sizeof(uint64_t) * nranks) != hipSuccess) {
    lego_set_error("lego_comm_create: stream / buffer allocation failed");
    return fail(LEGO_E_DEVICE);
  }
  c->sizes.assign(nranks, 0);
  c->offs.assign(nranks + 1, 0);
  *out = c;
  return LEGO_OK;
}

int lego_comm_set_timeout(lego_comm* c, int32_t timeout_ms) {
  if (!c || timeout_ms < 1) return LEGO_E_ARG;
  c->timeoutMs = timeout_ms;
  return LEGO_OK;
}

int lego_comm_count(lego_comm* c, int32_t* nranks) {
  if (!c || !nranks) return LEGO_E_ARG;
  if (!c->nc) {
    lego_set_error("lego_comm_count: the communicator was aborted");
    return LEGO_E_STATE;
  }
  int n = 0;
  COMM_NCCL(ncclCommCount(c->nc, &n));
  *nranks = n;
  return LEGO_OK;
}

int lego_comm_destroy(lego_comm* c) {
  delete c;
  return LEGO_OK;
}

static int comm_abort(lego_comm* c, bool inGroup, const char* what, const char* why) {
  if (inGroup) (void)ncclGroupEnd();
  lego_set_error("lego_comm: %s: %s (communicator aborted)", what, why);
  if (c->nc) (void)ncclCommAbort(c->nc);
  c->nc = nullptr;
  c->dead = true;
  c->haveResult = c->haveHost = false;
  return LEGO_E_DEVICE;
}
#define COMM_TRY_HIP(call, inGroup)                                          \
  do {                                                                      \
    hipError_t e_ = (call);                                                 \
    if (e_ != hipSuccess) return comm_abort(c, inGroup, #call, hipGetErrorString(e_)); \
  } while (0)
#define COMM_TRY_NCCL(call, inGroup)                                         \
  do {                                                                      \
    ncclResult_t r_ = (call);                                               \
    if (r_ != ncclSuccess) return comm_abort(c, inGroup, #call, ncclGetErrorString(r_)); \
  } while (0)

// Waits for the communicator's stream within c->timeoutMs: polls
// hipStreamQuery (a peer that never joins leaves the collective's kernel
// spinning, so an unbounded hipStreamSynchronize would never return).
static int comm_sync(lego_comm* c, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; ++spin) {
    const hipError_t e = hipStreamQuery(c->s);
    if (e == hipSuccess) return LEGO_OK;
    if (e != hipErrorNotReady) return comm_abort(c, false, what, hipGetErrorString(e));
    const auto ms =
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (ms > c->timeoutMs) {
      char why[96];
      std::snprintf(why, sizeof(why), "timed out after %lld ms (a peer never joined?)", (long long)ms);
      return comm_abort(c, false, what, why);
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

int lego_comm_gather_handoff_ex(lego_comm* c, lego_ctx* ctx, int32_t root, uint32_t flags) {
  if (!c || !ctx || root < 0 || root >= c->nranks || (flags & ~LEGO_COMM_DEVICE_RESULT)) return LEGO_E_ARG;
  if (c->dead) {
    lego_set_error("lego_comm: the communicator was aborted by an earlier error");
    return LEGO_E_STATE;
  }
  c->haveResult = c->haveHost = false;
  COMM_HIP(hipSetDevice(c->device));
  // the previous gather's send reads ctx's packet buffer, which the pack reuses
  if (comm_sync(c, "previous gather") != LEGO_OK) return LEGO_E_DEVICE;
  const void* pkt = nullptr;
  uint64_t bytes = 0;
  const int packSt = lego_handoff_pack(ctx, &pkt, &bytes);  // complete on return
  if (packSt != LEGO_OK) { pkt = nullptr; bytes = 0; }     // take part with an empty packet
  COMM_TRY_HIP(hipMemcpyAsync(c->dSize, &bytes, sizeof(bytes), hipMemcpyHostToDevice, c->s), false);
  COMM_TRY_NCCL(ncclGather(c->dSize, c->dSizes, 1, ncclUint64, root, c->nc, c->s), false);
  const bool isRoot = c->rank == root;
  if (isRoot) {
    COMM_TRY_HIP(hipMemcpyAsync(c->sizes.data(), c->dSizes, sizeof(uint64_t) * c->nranks, hipMemcpyDeviceToHost, c->s),
                 false);
    if (comm_sync(c, "ncclGather of the packet sizes") != LEGO_OK) return LEGO_E_DEVICE;
    for (int r = 0; r < c->nranks; ++r) c->offs[r + 1] = c->offs[r] + ((c->sizes[r] + 255) & ~(uint64_t)255);
    const size_t need = c->offs[c->nranks];
    if (need > c->recvCap) {
      if (c->dRecv) COMM_TRY_HIP(hipFree(c->dRecv), false);
      c->dRecv = nullptr;
      c->recvCap = 0;
      COMM_TRY_HIP(hipMalloc(&c->dRecv, need), false);
      c->recvCap = need;
    }
    if (bytes) COMM_TRY_HIP(hipMemcpyAsync(c->dRecv + c->offs[root], pkt, bytes, hipMemcpyDeviceToDevice, c->s), false);
  }
  COMM_TRY_NCCL(ncclGroupStart(), false);
  if (isRoot) {
    for (int r = 0; r < c->nranks; ++r)
      if (r != root && c->sizes[r])
        COMM_TRY_NCCL(ncclRecv(c->dRecv + c->offs[r], c->sizes[r], ncclUint8, r, c->nc, c->s), true);
  } else if (bytes) {
    COMM_TRY_NCCL(ncclSend(pkt, bytes, ncclUint8, root, c->nc, c->s), true);
  }
  COMM_TRY_NCCL(ncclGroupEnd(), false);
  // root copied its own packet on c->s too: either way the context's buffer is
  // read on c->s until this point of the stream
  if (bytes && lego_handoff_fence(ctx, c->s) != LEGO_OK) return comm_abort(c, false, "lego_handoff_fence", "event");
  if (!(flags & LEGO_COMM_DEVICE_RESULT)) {
    if (isRoot) {
      const size_t need = c->offs[c->nranks];
      if (need > c->hCap) {
        if (c->hRecv) COMM_TRY_HIP(hipHostFree(c->hRecv), false);
        c->hRecv = nullptr;
        c->hCap = 0;
        COMM_TRY_HIP(hipHostMalloc(&c->hRecv, need, hipHostMallocDefault), false);
        c->hCap = need;
      }
      COMM_TRY_HIP(hipMemcpyAsync(c->hRecv, c->dRecv, need, hipMemcpyDeviceToHost, c->s), false);
    }
    if (comm_sync(c, "packet transfer") != LEGO_OK) return LEGO_E_DEVICE;
    c->haveHost = isRoot;
  }
  c->haveResult = isRoot;
  return packSt;
}

int lego_comm_gather_handoff(lego_comm* c, lego_ctx* ctx, int32_t root) {
  return lego_comm_gather_handoff_ex(c, ctx, root, 0);
}

int lego_comm_abort(lego_comm* c) {
  if (!c) return LEGO_E_ARG;
  if (c->device >= 0) (void)hipSetDevice(c->device);
  if (c->nc) (void)ncclCommAbort(c->nc);  // cancels what is still queued on c->s
  c->nc = nullptr;
  c->dead = true;
  c->haveResult = c->haveHost = false;
  return LEGO_OK;
}

int lego_comm_wait(lego_comm* c) {
  if (!c) return LEGO_E_ARG;
  if (c->dead) return LEGO_E_STATE;
  COMM_HIP(hipSetDevice(c->device));
  return comm_sync(c, "lego_comm_wait");
}

int lego_comm_handoff_device(lego_comm* c, int32_t rank, const void** dpacket, uint64_t* bytes) {
  if (!c || !dpacket || !bytes || rank < 0 || rank >= c->nranks) return LEGO_E_ARG;
  if (!c->haveResult) {
    lego_set_error("lego_comm_handoff_device: no gathered result on this rank (root, after a gather)");
    return LEGO_E_STATE;
  }
  *dpacket = c->dRecv + c->offs[rank];
  *bytes = c->sizes[rank];
  return LEGO_OK;
}

int lego_comm_handoff(lego_comm* c, int32_t rank, const void** packet, uint64_t* bytes) {
  if (!c || !packet || !bytes || rank < 0 || rank >= c->nranks) return LEGO_E_ARG;
  if (!c->haveHost) {
    lego_set_error("lego_comm_handoff: no host result on this rank (root, after lego_comm_gather_handoff)");
    return LEGO_E_STATE;
  }
  *packet = c->hRecv + c->offs[rank];
  *bytes = c->sizes[rank];
  return LEGO_OK;
}

}  // extern "C"
