// lvk_split.h -- the layer split of SURVEY.md 8e inside the library.
//
// The reference runs all n_layer layers of llama_eval_internal (llama.cpp:927-1197) in
// one process on one device.  LLaMA-65B split over S GPUs keeps that API: stage s owns
// the contiguous layers [s*L/S, (s+1)*L/S) (weights + KV slice) on its own HIP device,
// stage 0 the token embeddings, stage S-1 the final norm + lm_head; the only exchange is
// the residual stream inpL, f32 [N][n_embd], from stage s to s+1.
//
// Two forms share the stage hand-off code:
//  * Split -- one process drives all S devices behind llama.h (llama_init_from_file with
//    LVK_SPLIT / LVK_SPLIT_DEVICES, or lvk_init_split): ncclCommInitAll over the S
//    devices and grouped ncclSend/ncclRecv of x on the stages' streams, so the host never
//    waits between hops; prompts are cut into micro-batches that flow through the stages
//    back to back (stage s runs micro-batch i+1 while stage s+1 runs i).  Stages that
//    share a device (one-GPU rehearsal) hand off with a stream-ordered device copy.
//  * StageLink -- one process per stage: lvk_stage_connect joins a ncclCommInitRank
//    communicator of S ranks (one GPU per rank), lvk_stage_connect_shm a host
//    shared-memory ring (any placement, several stages on one GPU included); then
//    lvk_stage_step does recv -> layers -> send on the rank's stream, plus the greedy token
//    relay from the last stage to the first.  A rank that fails after its first transfer
//    aborts the link (ncclCommAbort / the ring's abort word), so its peers fail instead of
//    waiting forever, and every wait of a stage step is bounded (LVK_STAGE_TIMEOUT_S).
#pragma once
#include <rccl/rccl.h>

#include <atomic>
#include <memory>
#include <string>

#include "lvk_context.h"

namespace lvk {

// RCCL entry points, resolved from librccl.so.1 on first use: the library does not link
// RCCL, only the rccl transport of a split loads it
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t *) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char * (*GetErrorString)(ncclResult_t) = nullptr;
    static const Rccl & get();   // throws lvk::Error when librccl cannot be loaded
    static bool available();     // librccl loads (no throw)
    void check(ncclResult_t r, const char * what) const;
};

// current HIP device for the lifetime of the guard
struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int dev);
    ~DeviceGuard();
};

// contiguous layer ranges: stage s owns [s*L/S, (s+1)*L/S)  (pipeline.py layer_ranges)
inline std::pair<int, int> stage_layers(int n_layer, int n_stages, int s) {
    return {s * n_layer / n_stages, (s + 1) * n_layer / n_stages};
}

struct Split {
    std::vector<std::unique_ptr<Context>> owned;   // stages 0..S-2 (S-1 is the llama_context's own)
    std::vector<Context *> st;                     // every stage in order
    std::vector<int> devices;
    bool rccl = false;                             // transport: RCCL send/recv, else device copies
    std::vector<ncclComm_t> comms;                 // rank s = stage s
    std::vector<hipEvent_t> ev_out, ev_in;         // copy transport: x of s ready / taken by s+1
    int micro = 64;                                // prompt micro-batch (tokens); 0 = whole batch

    ~Split();
    // after the stages exist: comms (distinct devices, unless transport "copy") or events
    void connect(const char * transport);
    void hop(int s, int n);
    void eval(const int * tokens, int n, int n_past, bool greedy = false);
    size_t kv_bytes() const;
    void kv_get(std::vector<uint8_t> & out) const;
    void kv_set(const uint8_t * src, size_t n);
};

// The point-to-point transport of a one-process-per-stage link.  send/recv move `bytes`
// between device buffers of neighbouring stages in the order of `stream` (RCCL: queued on
// the stream; shm: the host waits for the stream, then copies through the ring).
struct StageTransport {
    virtual ~StageTransport() = default;
    virtual const char * name() const = 0;
    virtual void send(const void * d, size_t bytes, int peer, hipStream_t s) = 0;
    virtual void recv(void * d, size_t bytes, int peer, hipStream_t s) = 0;
    // wait for the stream with the link's health check and time limit; throws on failure
    virtual void wait(hipStream_t s) = 0;
    // make every peer's pending and future waits on this link fail (no throw)
    virtual void abort() noexcept = 0;
};

struct StageLink {
    std::unique_ptr<StageTransport> t;
    int stage = 0, n_stages = 1;
};

// one RCCL communicator of S ranks (one GPU each)
std::unique_ptr<StageTransport> make_rccl_transport(const void * unique_id, int n_stages, int stage, int device);
// a POSIX shared-memory ring named `name` (every stage opens the same name; stage 0 creates
// it and unlinks the name once all stages have joined); messages of any size travel in
// 1 MiB pieces
std::unique_ptr<StageTransport> make_shm_transport(const char * name, int n_stages, int stage);
// seconds a stage step may wait on its link (LVK_STAGE_TIMEOUT_S, default 300)
double stage_timeout_s();

// lvk_stage_step: one eval of this rank's stage between its neighbours; returns the next
// greedy token on the first and last stage when greedy, else 0
int stage_step(Context & c, const int * tokens, int n, int n_past, bool greedy, int micro);
// the link alone: `iters` laps of a `bytes` message around the stage ring (stage 0 sends to 1,
// ..., the last stage back to 0), every stage taking part; returns microseconds per hop
double stage_link_probe(Context & c, size_t bytes, int iters);

}  // namespace lvk
