// lvk_split.cpp -- layer split over devices (lvk_split.h).
#include "lvk_split.h"

#include <dlfcn.h>

#include <cstring>
#include <mutex>

namespace lvk {

void SplitDel::operator()(Split * p) const { delete p; }
void StageLinkDel::operator()(StageLink * p) const { delete p; }

DeviceGuard::DeviceGuard(int dev) {
    LVK_HIP(hipGetDevice(&prev));
    if (dev != prev) LVK_HIP(hipSetDevice(dev));
}
DeviceGuard::~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void) hipSetDevice(prev);
}

const Rccl & Rccl::get() {
    static Rccl r;
    static std::string err;
    static std::once_flag once;
    std::call_once(once, [] {
        void * h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) { err = std::string("cannot load librccl.so.1: ") + dlerror(); return; }
        auto sym = [&](const char * n) {
            void * f = dlsym(h, n);
            if (!f && err.empty()) err = std::string("librccl.so.1 lacks ") + n;
            return f;
        };
        r.GetUniqueId = (decltype(r.GetUniqueId)) sym("ncclGetUniqueId");
        r.CommInitAll = (decltype(r.CommInitAll)) sym("ncclCommInitAll");
        r.CommInitRank = (decltype(r.CommInitRank)) sym("ncclCommInitRank");
        r.CommDestroy = (decltype(r.CommDestroy)) sym("ncclCommDestroy");
        r.Send = (decltype(r.Send)) sym("ncclSend");
        r.Recv = (decltype(r.Recv)) sym("ncclRecv");
        r.GroupStart = (decltype(r.GroupStart)) sym("ncclGroupStart");
        r.GroupEnd = (decltype(r.GroupEnd)) sym("ncclGroupEnd");
        r.GetErrorString = (decltype(r.GetErrorString)) sym("ncclGetErrorString");
    });
    if (!err.empty()) throw Error("llama.vk_amd: " + err);
    return r;
}

void Rccl::check(ncclResult_t res, const char * what) const {
    if (res != ncclSuccess) throw Error(std::string("llama.vk_amd: ") + what + ": " + GetErrorString(res));
}

// ---------------------------------------------------------------------------
// Split: one process, S devices
// ---------------------------------------------------------------------------
Split::~Split() {
    if (!comms.empty()) {
        const Rccl & R = Rccl::get();
        for (ncclComm_t c : comms)
            if (c) (void) R.CommDestroy(c);
    }
    for (hipEvent_t e : ev_out) if (e) (void) hipEventDestroy(e);
    for (hipEvent_t e : ev_in) if (e) (void) hipEventDestroy(e);
}

void Split::connect(const char * transport) {
    const int S = (int) st.size();
    bool distinct = true;
    for (int a = 0; a < S; ++a)
        for (int b = a + 1; b < S; ++b) distinct &= devices[a] != devices[b];
    const std::string t = transport ? transport : "";
    if (t == "rccl" && !distinct) throw Error("llama.vk_amd: the rccl split transport needs one device per stage");
    if (t != "" && t != "rccl" && t != "copy") throw Error("llama.vk_amd: LVK_SPLIT_TRANSPORT must be rccl or copy");
    rccl = S > 1 && distinct && t != "copy";
    if (rccl) {
        const Rccl & R = Rccl::get();
        comms.assign(S, nullptr);
        R.check(R.CommInitAll(comms.data(), S, devices.data()), "ncclCommInitAll");
        return;
    }
    ev_out.assign(S, nullptr);
    ev_in.assign(S, nullptr);
    for (int s = 0; s + 1 < S; ++s) {
        { DeviceGuard g(devices[s]); LVK_HIP(hipEventCreateWithFlags(&ev_out[s], hipEventDisableTiming)); }
        { DeviceGuard g(devices[s + 1]); LVK_HIP(hipEventCreateWithFlags(&ev_in[s], hipEventDisableTiming)); }
    }
}

// hand x [n][E] of stage s to stage s+1, stream-ordered on both sides: stage s+1's next
// kernels see it, and stage s overwrites its x only after it has left
void Split::hop(int s, int n) {
    Context & a = *st[s];
    Context & b = *st[s + 1];
    const size_t cnt = (size_t) n * a.model.hp.n_embd;
    if (rccl) {
        const Rccl & R = Rccl::get();
        R.check(R.GroupStart(), "ncclGroupStart");
        const ncclResult_t r1 = R.Send(a.x, cnt, ncclFloat32, s + 1, comms[s], a.stream);
        const ncclResult_t r2 = R.Recv(b.x, cnt, ncclFloat32, s, comms[s + 1], b.stream);
        const ncclResult_t r3 = R.GroupEnd();
        R.check(r1, "ncclSend");
        R.check(r2, "ncclRecv");
        R.check(r3, "ncclGroupEnd");
        return;
    }
    { DeviceGuard g(a.device); LVK_HIP(hipEventRecord(ev_out[s], a.stream)); }
    {
        DeviceGuard g(b.device);
        LVK_HIP(hipStreamWaitEvent(b.stream, ev_out[s], 0));
        LVK_HIP(hipMemcpyAsync(b.x, a.x, cnt * sizeof(float), hipMemcpyDeviceToDevice, b.stream));
        LVK_HIP(hipEventRecord(ev_in[s], b.stream));
    }
    { DeviceGuard g(a.device); LVK_HIP(hipStreamWaitEvent(a.stream, ev_in[s], 0)); }
}

// llama_eval over the stages: every slice (the whole call, or a prompt micro-batch) is
// enqueued stage after stage with the hand-offs in between; the host waits once, at the end
void Split::eval(const int * tokens, int n, int n_past, bool greedy) {
    const int S = (int) st.size();
    Context & last = *st.back();
    if (n <= 0 || n_past < 0 || n_past + n > last.n_ctx_user) throw Error("llama.vk_amd: n_past + n_tokens exceeds n_ctx");
    const int m = (micro > 0 && n > micro) ? micro : n;
    std::string err;
    try {
        for (int off = 0; off < n; off += m) {
            const int k = std::min(m, n - off);
            EvalPart p;
            p.tok_off = off;
            p.n_total = n;
            p.copy_out = off + k == n;
            p.head = p.copy_out || last.logits_all;   // last-token logits: only the final slice needs lm_head
            for (int s = 0; s < S; ++s) {
                DeviceGuard g(st[s]->device);
                EvalPart ps = p;
                ps.greedy = greedy && s == S - 1;
                st[s]->begin_eval(s == 0 ? tokens + off : nullptr, k, n_past + off, ps);
                if (s + 1 < S) hop(s, k);
            }
        }
    } catch (const Error & e) {
        err = e.msg;
    }
    // drain every stage (also after a failed enqueue), then report the first error
    for (int s = 0; s < S; ++s) {
        try {
            DeviceGuard g(st[s]->device);
            st[s]->end_eval(greedy && s == S - 1);
        } catch (const Error & e) {
            if (err.empty()) err = e.msg;
        }
    }
    if (!err.empty()) {
        last.logits_valid = false;
        throw Error(err);
    }
}

size_t Split::kv_bytes() const {
    size_t b = 0;
    for (const Context * c : st) b += c->kv_bytes();
    return b;
}

// the reference's KV bytes are K of every layer, then V of every layer (llama.cpp:1678-1701):
// stage halves concatenated in layer order
void Split::kv_get(std::vector<uint8_t> & out) const {
    out.resize(kv_bytes());
    const size_t half = out.size() / 2;
    size_t off = 0;
    for (const Context * c : st) {
        DeviceGuard g(c->device);
        const size_t h = c->kv_bytes() / 2;
        LVK_HIP(hipMemcpy(out.data() + off, c->kc, h, hipMemcpyDeviceToHost));
        LVK_HIP(hipMemcpy(out.data() + half + off, c->vc, h, hipMemcpyDeviceToHost));
        off += h;
    }
}

void Split::kv_set(const uint8_t * src, size_t n) {
    if (n != kv_bytes()) throw Error("llama_set_kv_cache: size mismatch");
    const size_t half = n / 2;
    size_t off = 0;
    for (Context * c : st) {
        DeviceGuard g(c->device);
        const size_t h = c->kv_bytes() / 2;
        LVK_HIP(hipMemcpy(c->kc, src + off, h, hipMemcpyHostToDevice));
        LVK_HIP(hipMemcpy(c->vc, src + half + off, h, hipMemcpyHostToDevice));
        off += h;
    }
}

// ---------------------------------------------------------------------------
// StageLink: one process per stage
// ---------------------------------------------------------------------------
StageLink::~StageLink() {
    if (comm) (void) Rccl::get().CommDestroy(comm);
}

int stage_step(Context & c, const int * tokens, int n, int n_past, bool greedy, int micro) {
    const Rccl & R = Rccl::get();
    if (!c.link) throw Error("llama.vk_amd: stage not connected (lvk_stage_connect)");
    StageLink & L = *c.link;
    const int s = L.stage, S = L.n_stages;
    if (greedy && n != 1) throw Error("llama.vk_amd: a greedy stage step takes one token");
    if (n <= 0 || n_past < 0 || n_past + n > c.n_ctx_user) throw Error("llama.vk_amd: n_past + n_tokens exceeds n_ctx");
    const int m = (micro > 0 && n > micro) ? micro : n;
    const size_t E = c.model.hp.n_embd;
    DeviceGuard g(c.device);
    std::string err;
    try {
        for (int off = 0; off < n; off += m) {
            const int k = std::min(m, n - off);
            EvalPart p;
            p.tok_off = off;
            p.n_total = n;
            p.copy_out = off + k == n;
            p.head = p.copy_out || c.logits_all;
            p.greedy = greedy && s == S - 1;
            if (s > 0) R.check(R.Recv(c.x, (size_t) k * E, ncclFloat32, s - 1, L.comm, c.stream), "ncclRecv");
            c.begin_eval(s == 0 ? tokens + off : nullptr, k, n_past + off, p);
            if (s + 1 < S) R.check(R.Send(c.x, (size_t) k * E, ncclFloat32, s + 1, L.comm, c.stream), "ncclSend");
        }
        // greedy decode: the last stage's device argmax goes straight to the first stage,
        // whose host needs it to embed the next token
        if (greedy && S > 1) {
            if (s == S - 1) R.check(R.Send(c.greedy_d, 1, ncclInt32, 0, L.comm, c.stream), "ncclSend");
            if (s == 0) {
                R.check(R.Recv(c.greedy_d, 1, ncclInt32, S - 1, L.comm, c.stream), "ncclRecv");
                LVK_HIP(hipMemcpyAsync(c.greedy_h, c.greedy_d, sizeof(int), hipMemcpyDeviceToHost, c.stream));
            }
        }
    } catch (const Error & e) {
        err = e.msg;
    }
    try {
        c.end_eval(greedy && s == S - 1);
    } catch (const Error & e) {
        if (err.empty()) err = e.msg;
    }
    if (!err.empty()) throw Error(err);
    return greedy && (s == 0 || s == S - 1) ? *c.greedy_h : 0;
}

}  // namespace lvk
