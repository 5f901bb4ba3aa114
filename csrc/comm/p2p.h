// Native stage-to-stage data plane over RCCL (csrc/comm/p2p.cpp).
//
// A channel is one RCCL communicator (a peer pair, or a 1-rank loopback) with
// its own high-priority HIP transfer stream and a ring of completion events.
// Ops are posted either on the channel stream — ordered after the work the
// caller's stream had queued at post time, completion returned as a token the
// caller's stream can wait on without blocking the host — or directly on the
// caller's stream (HIP graph capture: the hop becomes graph nodes next to the
// stage's kernels).
#pragma once
#include <hip/hip_runtime.h>

extern "C" {
// 1 if librccl could be resolved in this process (torch's copy when loaded).
int dnn_comm_available();
// Last error message of this thread's comm calls ("" if none).
const char* dnn_comm_last_error();
// 128-byte RCCL unique id (the rendezvous token the lowest rank publishes).
int dnn_comm_unique_id(void* out128);
// New channel (returns an opaque handle, 0 on failure).  async = 1: the
// (blocking, collective) communicator init runs on a background thread, so a
// rank can create all its pair channels in any order without deadlocking on
// a peer that creates them in another order; ops wait for it.
long long dnn_comm_create(const void* id128, int nranks, int rank, int device, int async);
// Wait for the init: 0 ready, 1 still pending after timeout_ms, < 0 failed.
int dnn_comm_wait_ready(long long h, int timeout_ms);
// Post one op: kind 0 = send, 1 = recv.  on_stream = 0: on the channel stream
// (returns a token > 0), 1: directly on st (returns 0).  < 0 on error.
long long dnn_comm_post(long long h, int kind, void* ptr, long long bytes, int peer, hipStream_t st, int on_stream);
// Several ops in one RCCL group (concurrent; the only legal form of a send to
// self), same stream modes and return as dnn_comm_post.
long long dnn_comm_group(long long h, int n, const int* kinds, void* const* ptrs, const long long* bytes,
                         const int* peers, hipStream_t st, int on_stream);
// Make st wait (device side) for the op of token.
int dnn_comm_wait(long long h, long long token, hipStream_t st);
// 1 if the op of token completed, 0 if pending, < 0 on an async RCCL error.
int dnn_comm_query(long long h, long long token);
// Host wait with a deadline: 0 done, 1 timeout, < 0 async RCCL error.
int dnn_comm_sync(long long h, long long token, int timeout_ms);
// Async RCCL error of the communicator (0 = none).
int dnn_comm_async_error(long long h);
// Abort: in-flight RCCL kernels of this channel return (peer died / watchdog).
int dnn_comm_abort(long long h);
// Destroy (after every op completed or the channel was aborted).
int dnn_comm_destroy(long long h);
// Byte / op counters of a channel: out[0..3] = sent ops, sent bytes, recv ops, recv bytes.
int dnn_comm_stats(long long h, long long* out4);
}
