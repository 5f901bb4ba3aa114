// Native stage-to-stage data plane over RCCL: see p2p.h for the contract.
//
// Why a module of our own instead of torch.distributed's isend/irecv (which
// the gloo paths still use): ProcessGroupNCCL creates a peer pair's
// communicator lazily and blockingly inside the first op (two stages that
// open their links in different orders can deadlock there), wraps every op in
// a Work object with its own events and host-side bookkeeping, and cannot put
// a hop inside a HIP graph.  Here
//   * every pair channel is created eagerly and its collective init runs on a
//     background thread (any creation order is deadlock-free; the id is
//     published through the process group's TCP store by the lower rank);
//   * an op posted on the channel's own high-priority stream is ordered after
//     the work the caller's stream had queued when it was posted (the buffer
//     is complete / free), and its completion is an event of a fixed ring that
//     the caller's stream waits on device-side — the host never blocks on a
//     hop;
//   * an op posted on the caller's stream instead is plain stream work, so a
//     stage step can capture recv -> kernels -> send as one HIP graph;
//   * abort makes in-flight RCCL kernels of the channel return, so the
//     failure watchdog (parallel/watchdog.py) can tear a stage down without
//     leaving a P2P kernel spinning on the GPU.
// librccl is resolved at run time (dlopen of the copy torch already loaded —
// same soname — else the ROCm one), so the kernel library builds and loads
// without it; rccl.h supplies the types only.
//
// Reference behaviour replaced: the per-request gRPC channel + protobuf
// serialisation hop of node.py:45-55,73-89.
#include "comm/p2p.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

namespace dnn {
namespace comm {

struct Api {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  bool ok = false;
  std::string why;
};

thread_local std::string g_err;

static int fail(const std::string& msg, int rc = -1) {
  g_err = msg;
  return rc;
}

template <typename F>
static bool sym(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  return f != nullptr;
}

static const Api& api() {
  static Api a = [] {
    Api r;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, if loaded
    if (h == nullptr) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) {
      r.why = std::string("librccl.so.1 not loadable: ") + dlerror();
      return r;
    }
    r.ok = sym(h, "ncclGetUniqueId", r.GetUniqueId) && sym(h, "ncclCommInitRank", r.CommInitRank) &&
           sym(h, "ncclCommDestroy", r.CommDestroy) && sym(h, "ncclCommAbort", r.CommAbort) &&
           sym(h, "ncclCommGetAsyncError", r.CommGetAsyncError) && sym(h, "ncclGetErrorString", r.GetErrorString) &&
           sym(h, "ncclSend", r.Send) && sym(h, "ncclRecv", r.Recv) && sym(h, "ncclGroupStart", r.GroupStart) &&
           sym(h, "ncclGroupEnd", r.GroupEnd);
    if (!r.ok) r.why = "librccl.so.1 lacks a required symbol";
    return r;
  }();
  return a;
}

static std::string rccl_msg(const char* what, ncclResult_t rc) {
  return std::string(what) + ": " + (api().GetErrorString ? api().GetErrorString(rc) : "rccl error") + " (" +
         std::to_string((int)rc) + ")";
}

// Switches to a device for the scope (HIP's current device is per thread).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) hipSetDevice(prev);
  }
};

struct Channel {
  static constexpr int RING = 1024;  // completion events in flight per channel
  int nranks = 0, rank = 0, device = 0;
  // ops (post / group), abort's ncclCommAbort and destroy serialise on this;
  // abort only *tries* it for a bounded time (a post can be stuck waiting on a
  // dead peer's slot: it polls `aborted` and gives the lock back)
  std::timed_mutex mu;
  std::mutex join_mu;  // joining the init thread (several threads may ask)
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t in_ev[RING];
  hipEvent_t done_ev[RING];
  long long done_tok[RING];
  long long seq = 0;
  std::thread init;
  std::atomic<int> state{0};  // 0 pending, 1 ready, < 0 failed (-rc)
  std::string init_err;
  std::atomic<bool> aborted{false};
  std::atomic<bool> init_detached{false};  // abort left a blocked init running: never delete this Channel
  long long sent_ops = 0, sent_bytes = 0, recv_ops = 0, recv_bytes = 0;
};

static Channel* ch(long long h) { return reinterpret_cast<Channel*>(static_cast<uintptr_t>(h)); }

static int ensure_ready(Channel* c, int timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  while (c->state.load(std::memory_order_acquire) == 0) {
    if (c->aborted.load()) return fail("channel aborted during communicator init", -3);
    if (timeout_ms >= 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
      return 1;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  {
    std::lock_guard<std::mutex> j(c->join_mu);
    if (c->init.joinable() && !c->init_detached.load()) c->init.join();
  }
  if (c->state.load() < 0) return fail("rccl communicator init failed: " + c->init_err, -2);
  if (c->aborted.load()) return fail("channel was aborted", -3);
  return 0;
}

static int slot_timeout_ms() {
  static const int ms = [] {
    const char* e = std::getenv("DNN_RCCL_SLOT_TIMEOUT_MS");
    return e ? std::atoi(e) : 300000;
  }();
  return ms;
}

// Claim the next ring slot (the op that used it before must have completed).
// The wait for that op is a bounded poll, never hipEventSynchronize: a peer
// that died with ops in flight must surface as an error (or an abort from the
// watchdog thread), not as a host thread blocked forever.
static int next_slot(Channel* c, long long& tok) {
  const long long want = c->seq + 1;
  const int s = (int)(want % Channel::RING);
  if (c->done_tok[s] != 0) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipEventQuery(c->done_ev[s]);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) return fail(std::string("event query: ") + hipGetErrorString(e));
      if (c->aborted.load()) return fail("channel was aborted", -3);
      if (c->comm != nullptr) {
        ncclResult_t ae = ncclSuccess;
        api().CommGetAsyncError(c->comm, &ae);
        if (ae != ncclSuccess && ae != ncclInProgress) return fail(rccl_msg("rccl async error", ae));
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(slot_timeout_ms()))
        return fail("completion ring full: op " + std::to_string(c->done_tok[s]) + " not complete after " +
                    std::to_string(slot_timeout_ms()) + " ms (peer dead?)");
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  tok = c->seq = want;
  c->done_tok[s] = tok;
  return s;
}

static ncclResult_t issue(Channel* c, int kind, void* ptr, long long bytes, int peer, hipStream_t st) {
  if (kind == 0) {
    c->sent_ops += 1;
    c->sent_bytes += bytes;
    return api().Send(ptr, (size_t)bytes, ncclUint8, peer, c->comm, st);
  }
  c->recv_ops += 1;
  c->recv_bytes += bytes;
  return api().Recv(ptr, (size_t)bytes, ncclUint8, peer, c->comm, st);
}

// Shared body of post / group: n ops in one RCCL group if n > 1.
static long long post_ops(long long h, int n, const int* kinds, void* const* ptrs, const long long* bytes,
                          const int* peers, hipStream_t st, int on_stream) {
  Channel* c = ch(h);
  if (c == nullptr) return fail("null channel");
  // never block on the init here: Python waits for it with
  // dnn_comm_wait_ready, GIL released, before a channel's first op
  if (int r = ensure_ready(c, 0)) return r == 1 ? fail("channel init still pending", -4) : r;
  std::lock_guard<std::timed_mutex> lock(c->mu);
  if (c->aborted.load() || c->comm == nullptr) return fail("channel was aborted", -3);
  for (int i = 0; i < n; ++i) {
    if (kinds[i] != 0 && kinds[i] != 1) return fail("op kind must be 0 (send) or 1 (recv)");
    if (peers[i] < 0 || peers[i] >= c->nranks) return fail("peer " + std::to_string(peers[i]) + " out of range");
    if (bytes[i] < 0 || (bytes[i] > 0 && ptrs[i] == nullptr)) return fail("bad buffer");
  }
  DeviceGuard g(c->device);
  hipStream_t run = on_stream ? st : c->stream;
  long long tok = 0;
  int slot = -1;
  if (!on_stream) {
    slot = next_slot(c, tok);
    if (slot < 0) return slot;
    // the transfer reads / overwrites its buffer only after the work the
    // caller queued before posting it
    if (hipEventRecord(c->in_ev[slot], st) != hipSuccess || hipStreamWaitEvent(c->stream, c->in_ev[slot], 0) != hipSuccess)
      return fail("ordering the channel stream after the caller's stream failed");
  }
  ncclResult_t rc = ncclSuccess;
  if (n > 1) rc = api().GroupStart();
  for (int i = 0; i < n && rc == ncclSuccess; ++i) rc = issue(c, kinds[i], ptrs[i], bytes[i], peers[i], run);
  if (n > 1) {
    const ncclResult_t rc2 = api().GroupEnd();
    if (rc == ncclSuccess) rc = rc2;
  }
  if (rc != ncclSuccess) return fail(rccl_msg(n > 1 ? "rccl group" : "rccl p2p", rc));
  if (!on_stream) {
    if (hipEventRecord(c->done_ev[slot], c->stream) != hipSuccess) return fail("recording the completion event failed");
    return tok;
  }
  return 0;
}

}  // namespace comm
}  // namespace dnn

using namespace dnn::comm;

extern "C" {

int dnn_comm_available() { return api().ok ? 1 : 0; }

const char* dnn_comm_last_error() { return g_err.c_str(); }

int dnn_comm_unique_id(void* out128) {
  if (!api().ok) return fail(api().why);
  ncclUniqueId id;
  const ncclResult_t rc = api().GetUniqueId(&id);
  if (rc != ncclSuccess) return fail(rccl_msg("ncclGetUniqueId", rc));
  std::memcpy(out128, &id, sizeof(id));
  return 0;
}

long long dnn_comm_create(const void* id128, int nranks, int rank, int device, int async) {
  if (!api().ok) return fail(api().why, 0);
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail("bad rank / nranks", 0);
  auto* c = new Channel();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  std::memset(c->done_tok, 0, sizeof(c->done_tok));
  {
    DeviceGuard g(device);
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);  // hi = numerically smallest = most urgent
    bool ok = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi) == hipSuccess;
    for (int i = 0; ok && i < Channel::RING; ++i)
      ok = hipEventCreateWithFlags(&c->in_ev[i], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&c->done_ev[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      delete c;
      return fail("stream / event creation failed", 0);
    }
  }
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  auto body = [c, id]() {
    hipSetDevice(c->device);
    const ncclResult_t rc = api().CommInitRank(&c->comm, c->nranks, id, c->rank);
    if (rc != ncclSuccess) {
      c->init_err = rccl_msg("ncclCommInitRank", rc);
      c->state.store(-(int)rc - 1, std::memory_order_release);
    } else {
      c->state.store(1, std::memory_order_release);
    }
  };
  if (async)
    c->init = std::thread(body);
  else
    body();
  return static_cast<long long>(reinterpret_cast<uintptr_t>(c));
}

int dnn_comm_wait_ready(long long h, int timeout_ms) {
  Channel* c = ch(h);
  if (c == nullptr) return fail("null channel");
  return ensure_ready(c, timeout_ms);
}

long long dnn_comm_post(long long h, int kind, void* ptr, long long bytes, int peer, hipStream_t st, int on_stream) {
  return post_ops(h, 1, &kind, &ptr, &bytes, &peer, st, on_stream);
}

long long dnn_comm_group(long long h, int n, const int* kinds, void* const* ptrs, const long long* bytes,
                         const int* peers, hipStream_t st, int on_stream) {
  if (n < 1) return fail("empty group");
  return post_ops(h, n, kinds, ptrs, bytes, peers, st, on_stream);
}

int dnn_comm_wait(long long h, long long token, hipStream_t st) {
  Channel* c = ch(h);
  if (c == nullptr || token <= 0 || token > c->seq) return fail("bad token");
  const int s = (int)(token % Channel::RING);
  if (c->done_tok[s] != token) return 0;  // the slot was reused: its op completed long ago
  return hipStreamWaitEvent(st, c->done_ev[s], 0) == hipSuccess ? 0 : fail("stream wait failed");
}

int dnn_comm_async_error(long long h) {
  Channel* c = ch(h);
  if (c == nullptr || c->comm == nullptr) return 0;
  ncclResult_t e = ncclSuccess;
  api().CommGetAsyncError(c->comm, &e);
  return (int)e;
}

int dnn_comm_query(long long h, long long token) {
  Channel* c = ch(h);
  if (c == nullptr || token <= 0 || token > c->seq) return fail("bad token");
  const int s = (int)(token % Channel::RING);
  if (c->done_tok[s] != token) return 1;
  const hipError_t e = hipEventQuery(c->done_ev[s]);
  if (e == hipSuccess) return 1;
  if (e != hipErrorNotReady) return fail(std::string("event query: ") + hipGetErrorString(e));
  if (int ae = dnn_comm_async_error(h)) return fail(rccl_msg("rccl async error", (ncclResult_t)ae));
  return 0;
}

int dnn_comm_sync(long long h, long long token, int timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const int q = dnn_comm_query(h, token);
    if (q != 0) return q == 1 ? 0 : q;
    if (timeout_ms >= 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return 1;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

int dnn_comm_abort(long long h) {
  Channel* c = ch(h);
  if (c == nullptr) return 0;
  const bool was = c->aborted.exchange(true);  // a post waiting on a slot sees this and returns
  {
    std::lock_guard<std::mutex> j(c->join_mu);
    if (c->state.load() == 0) {  // init still blocked on a peer that may be dead: leave it, never join
      if (c->init.joinable()) {
        c->init.detach();
        c->init_detached.store(true);
      }
      return 0;
    }
    if (c->init.joinable() && !c->init_detached.load()) c->init.join();
  }
  std::unique_lock<std::timed_mutex> lock(c->mu, std::defer_lock);
  if (!was && lock.try_lock_for(std::chrono::seconds(5)) && c->comm != nullptr) {
    api().CommAbort(c->comm);
    c->comm = nullptr;
  }
  return 0;
}

int dnn_comm_destroy(long long h) {
  Channel* c = ch(h);
  if (c == nullptr) return 0;
  {
    std::lock_guard<std::mutex> j(c->join_mu);
    if (c->state.load() == 0 && !c->init.joinable()) c->init_detached.store(true);
    if (c->init_detached.load()) return 0;  // its init thread may still write into it: leak, never free
    if (c->init.joinable()) c->init.join();
  }
  std::lock_guard<std::timed_mutex> lock(c->mu);
  int rc = 0;
  {
    DeviceGuard g(c->device);
    if (c->comm != nullptr && !c->aborted) {
      hipStreamSynchronize(c->stream);
      const ncclResult_t r = api().CommDestroy(c->comm);
      if (r != ncclSuccess) rc = fail(rccl_msg("ncclCommDestroy", r));
    }
    for (int i = 0; i < Channel::RING; ++i) {
      hipEventDestroy(c->in_ev[i]);
      hipEventDestroy(c->done_ev[i]);
    }
    hipStreamDestroy(c->stream);
  }
  delete c;
  return rc;
}

int dnn_comm_stats(long long h, long long* out4) {
  Channel* c = ch(h);
  if (c == nullptr) return fail("null channel");
  out4[0] = c->sent_ops;
  out4[1] = c->sent_bytes;
  out4[2] = c->recv_ops;
  out4[3] = c->recv_bytes;
  return 0;
}

}  // extern "C"
