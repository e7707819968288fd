// loopback_rccl.cpp -- an in-process stand-in for RCCL's point-to-point API, for tests only.
//
// libptx.so dlopens RCCL (pathtracerdemo_amd/csrc/ptx_comm.cpp) and uses ncclGetUniqueId,
// ncclCommInitRank[Config] / InitAll, grouped ncclSend / ncclRecv, GetAsyncError, Finalize,
// Destroy and Abort.  With PTX_RCCL_LIB pointing at this library, several band handles of ONE
// process on ONE GPU run that exact code -- the static halo, the motion halo, pipelined frames,
// the neighbour check, the failure paths -- which real RCCL refuses (one rank per device).
// SURVEY.md §4 item 6 (a fake communicator so the exchange logic is testable without 8 GPUs).
//
// Semantics.  Every communicator belongs to a clique (one unique id).  ncclSend / ncclRecv record
// an event on their stream when posted (the data is ready there) and are queued per thread until
// the outermost ncclGroupEnd (an op outside a group is a group of one).  At ncclGroupEnd the
// thread adds its ops to the clique's pending set and matches every send (src -> dst, n-th on that
// channel) with the recv (dst <- src, n-th): for a matched pair the receiver's stream waits for the
// send's event, copies the bytes device to device and records `done`, and the sender's stream
// waits for `done` -- so each side's later work is ordered after the transfer, as with RCCL's
// blocking-for-the-GPU send / recv.  ncclGroupEnd then blocks (the host thread) until all of its
// own ops are matched: ranks driven from different host threads rendezvous like processes, and
// one thread may post every rank's ops in a single group (ptx_render_bands).  An op still
// unmatched after LOOPBACK_TIMEOUT_MS (default 20000) fails the group with ncclSystemError and
// marks the communicator's async error (a rank whose peer never renders).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

struct ncclComm {
    std::string clique;
    int nranks = 0, rank = 0;
    ncclResult_t error = ncclSuccess;
    std::map<int, uint64_t> sent, received;  // ops posted per peer (channel sequence numbers)
};

namespace {

struct Op {
    bool send = false;
    ncclComm *comm = nullptr;
    int peer = 0;
    void *ptr = nullptr;
    size_t bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ready = nullptr;  // send: the data is complete on the sender's stream
    uint64_t seq = 0;
    bool done = false;
    bool failed = false;
};

std::mutex g_mu;
std::condition_variable g_cv;
std::vector<std::shared_ptr<Op>> g_pending;  // posted by a group end, not matched yet
uint64_t g_next_id = 1;
int g_destroys = 0, g_aborts = 0, g_finalizes = 0, g_groups = 0, g_pairs = 0;
size_t g_bytes = 0;

thread_local int t_depth = 0;
thread_local std::vector<std::shared_ptr<Op>> t_ops;

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

int timeout_ms() {
    const char *e = std::getenv("LOOPBACK_TIMEOUT_MS");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 20000;
}

// (under g_mu) match every pending send with its recv and enqueue the transfers
ncclResult_t match_locked() {
    for (size_t i = 0; i < g_pending.size(); ++i) {
        Op &s = *g_pending[i];
        if (!s.send || s.done) continue;
        for (size_t j = 0; j < g_pending.size(); ++j) {
            Op &r = *g_pending[j];
            if (r.send || r.done || r.comm->clique != s.comm->clique || r.comm->rank != s.peer ||
                r.peer != s.comm->rank || r.seq != s.seq)
                continue;
            if (r.bytes != s.bytes) {
                s.failed = r.failed = true;
                s.done = r.done = true;
                s.comm->error = r.comm->error = ncclInvalidUsage;
                break;
            }
            hipEvent_t fin = nullptr;
            if (hipStreamWaitEvent(r.stream, s.ready, 0) != hipSuccess ||
                (s.bytes && hipMemcpyAsync(r.ptr, s.ptr, s.bytes, hipMemcpyDeviceToDevice, r.stream) != hipSuccess) ||
                hipEventCreateWithFlags(&fin, hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(fin, r.stream) != hipSuccess || hipStreamWaitEvent(s.stream, fin, 0) != hipSuccess) {
                s.failed = r.failed = true;
                s.comm->error = r.comm->error = ncclUnhandledCudaError;
            }
            if (fin) (void)hipEventDestroy(fin);  // (released once it has fired)
            s.done = r.done = true;
            ++g_pairs;
            g_bytes += s.bytes;
            break;
        }
    }
    std::vector<std::shared_ptr<Op>> left;
    for (auto &o : g_pending)
        if (!o->done) left.push_back(o);
    g_pending.swap(left);
    return ncclSuccess;
}

ncclResult_t post(bool send, void *ptr, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                  hipStream_t stream) {
    if (!comm || peer < 0 || peer >= comm->nranks || peer == comm->rank) return ncclInvalidArgument;
    const size_t tb = type_bytes(dt);
    if (!tb) return ncclInvalidArgument;
    auto op = std::make_shared<Op>();
    op->send = send;
    op->comm = comm;
    op->peer = peer;
    op->ptr = ptr;
    op->bytes = count * tb;
    op->stream = stream;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        op->seq = send ? comm->sent[peer]++ : comm->received[peer]++;
    }
    if (send) {
        if (hipEventCreateWithFlags(&op->ready, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(op->ready, stream) != hipSuccess)
            return ncclUnhandledCudaError;
    }
    t_ops.push_back(op);  // (ncclSend / ncclRecv open a group around every post)
    return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth > 0) --t_depth;
    if (t_depth > 0) return ncclSuccess;
    std::vector<std::shared_ptr<Op>> mine;
    mine.swap(t_ops);
    if (mine.empty()) return ncclSuccess;
    std::unique_lock<std::mutex> lk(g_mu);
    ++g_groups;
    for (auto &o : mine) g_pending.push_back(o);
    match_locked();
    g_cv.notify_all();
    auto all_done = [&] {
        for (auto &o : mine)
            if (!o->done) return false;
        return true;
    };
    const bool ok = g_cv.wait_for(lk, std::chrono::milliseconds(timeout_ms()), all_done);
    ncclResult_t rc = ncclSuccess;
    if (!ok) {  // a peer never posted its side: fail this group, drop its unmatched ops
        for (auto &o : mine)
            if (!o->done) {
                o->done = o->failed = true;
                o->comm->error = ncclSystemError;
            }
        std::vector<std::shared_ptr<Op>> left;
        for (auto &o : g_pending)
            if (!o->done) left.push_back(o);
        g_pending.swap(left);
        rc = ncclSystemError;
    }
    for (auto &o : mine) {
        if (o->failed && rc == ncclSuccess) rc = o->comm->error;
        if (o->ready) (void)hipEventDestroy(o->ready);
        o->ready = nullptr;
    }
    return rc;
}

ncclResult_t ncclSend(const void *sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    ncclGroupStart();
    const ncclResult_t r = post(true, const_cast<void *>(sendbuff), count, datatype, peer, comm, stream);
    const ncclResult_t e = ncclGroupEnd();
    return r != ncclSuccess ? r : e;
}

ncclResult_t ncclRecv(void *recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    ncclGroupStart();
    const ncclResult_t r = post(false, recvbuff, count, datatype, peer, comm, stream);
    const ncclResult_t e = ncclGroupEnd();
    return r != ncclSuccess ? r : e;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof *id);
    std::lock_guard<std::mutex> lk(g_mu);
    std::snprintf(id->internal, sizeof id->internal, "loopback-%llu",
                  (unsigned long long)(g_next_id++ + 1000003ull * (unsigned long long)std::rand()));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    auto *c = new ncclComm;
    c->clique.assign(id.internal, strnlen(id.internal, sizeof id.internal));
    c->nranks = nranks;
    c->rank = rank;
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank, ncclConfig_t *) {
    return ncclCommInitRank(comm, nranks, id, rank);
}

ncclResult_t ncclCommInitAll(ncclComm_t *comms, int ndev, const int *) {
    ncclUniqueId id;
    ncclGetUniqueId(&id);
    for (int i = 0; i < ndev; ++i)
        if (ncclResult_t r = ncclCommInitRank(comms + i, ndev, id, i)) return r;
    return ncclSuccess;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t *err) {
    if (!comm || !err) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_mu);
    *err = comm->error;
    return ncclSuccess;
}

ncclResult_t ncclCommFinalize(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_mu);
    ++g_finalizes;
    return comm->error;
}

static ncclResult_t release(ncclComm_t comm, int &counter) {
    if (!comm) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_mu);
    std::vector<std::shared_ptr<Op>> left;
    for (auto &o : g_pending)
        if (o->comm != comm) left.push_back(o);
    g_pending.swap(left);
    ++counter;
    delete comm;
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) { return release(comm, g_destroys); }
ncclResult_t ncclCommAbort(ncclComm_t comm) { return release(comm, g_aborts); }

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
    case ncclSuccess: return "no error (loopback)";
    case ncclSystemError: return "loopback: a peer never posted its side of the group";
    case ncclInvalidUsage: return "loopback: send and recv sizes differ";
    case ncclInvalidArgument: return "loopback: invalid argument";
    case ncclUnhandledCudaError: return "loopback: a HIP call failed";
    default: return "loopback: error";
    }
}

// test introspection: {groups, matched pairs, bytes moved, destroys, aborts, finalizes}
void loopback_stats(unsigned long long out[6]) {
    std::lock_guard<std::mutex> lk(g_mu);
    out[0] = (unsigned long long)g_groups;
    out[1] = (unsigned long long)g_pairs;
    out[2] = (unsigned long long)g_bytes;
    out[3] = (unsigned long long)g_destroys;
    out[4] = (unsigned long long)g_aborts;
    out[5] = (unsigned long long)g_finalizes;
}

}  // extern "C"
