// lvk_split.cpp -- layer split over devices (lvk_split.h).
#include "lvk_split.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

namespace lvk {

void SplitDel::operator()(Split * p) const { delete p; }
void StageLinkDel::operator()(StageLink * p) const { delete p; }

double stage_timeout_s() {
    const char * e = getenv("LVK_STAGE_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : 300.0;
}

DeviceGuard::DeviceGuard(int dev) {
    LVK_HIP(hipGetDevice(&prev));
    if (dev != prev) LVK_HIP(hipSetDevice(dev));
}
DeviceGuard::~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void) hipSetDevice(prev);
}

static std::string & rccl_err() {
    static std::string err;
    return err;
}

static Rccl & rccl_load() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        std::string & err = rccl_err();
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
        r.CommAbort = (decltype(r.CommAbort)) sym("ncclCommAbort");
        r.CommGetAsyncError = (decltype(r.CommGetAsyncError)) sym("ncclCommGetAsyncError");
        r.Send = (decltype(r.Send)) sym("ncclSend");
        r.Recv = (decltype(r.Recv)) sym("ncclRecv");
        r.GroupStart = (decltype(r.GroupStart)) sym("ncclGroupStart");
        r.GroupEnd = (decltype(r.GroupEnd)) sym("ncclGroupEnd");
        r.GetErrorString = (decltype(r.GetErrorString)) sym("ncclGetErrorString");
    });
    return r;
}

const Rccl & Rccl::get() {
    const Rccl & r = rccl_load();
    if (!rccl_err().empty()) throw Error("llama.vk_amd: " + rccl_err());
    return r;
}

bool Rccl::available() {
    rccl_load();
    return rccl_err().empty();
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
    if (rccl && t.empty() && !Rccl::available()) {
        // no transport asked for and no librccl: the stream-ordered device copies work
        // between distinct devices too (peer access or staged by the runtime)
        fprintf(stderr, "llama.vk_amd: librccl.so.1 not loadable, the split hands off by device copies\n");
        rccl = false;
    }
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
namespace {

using Clock = std::chrono::steady_clock;

double since_s(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// RCCL: ncclSend / ncclRecv on the stage stream; waits poll the stream and the
// communicator's asynchronous error, and a failure or the time limit aborts the
// communicator (its kernels stop, the peers' operations error out)
struct RcclTransport final : StageTransport {
    ncclComm_t comm = nullptr;
    const char * name() const override { return "rccl"; }
    ~RcclTransport() override {
        if (comm) (void) Rccl::get().CommDestroy(comm);
    }
    void send(const void * d, size_t bytes, int peer, hipStream_t s) override {
        const Rccl & R = Rccl::get();
        if (!comm) throw Error("llama.vk_amd: stage link aborted");
        R.check(R.Send(d, bytes, ncclInt8, peer, comm, s), "ncclSend");
    }
    void recv(void * d, size_t bytes, int peer, hipStream_t s) override {
        const Rccl & R = Rccl::get();
        if (!comm) throw Error("llama.vk_amd: stage link aborted");
        R.check(R.Recv(d, bytes, ncclInt8, peer, comm, s), "ncclRecv");
    }
    void wait(hipStream_t s) override {
        const Rccl & R = Rccl::get();
        const double limit = stage_timeout_s();
        const auto t0 = Clock::now();
        for (int i = 0;; ++i) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) return;
            if (q != hipErrorNotReady) LVK_HIP(q);
            ncclResult_t ae = ncclSuccess;
            if (comm && R.CommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                const std::string msg = std::string("llama.vk_amd: stage link RCCL error: ") + R.GetErrorString(ae);
                abort();
                throw Error(msg);
            }
            if (since_s(t0) > limit) {
                abort();
                throw Error("llama.vk_amd: stage step exceeded LVK_STAGE_TIMEOUT_S waiting for its neighbours");
            }
            if (i > 256) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    void abort() noexcept override {
        if (!comm) return;
        (void) Rccl::get().CommAbort(comm);
        comm = nullptr;
    }
};

// Host shared-memory ring (POSIX shm, every stage opens the same name): ring s carries
// stage s -> (s + 1) % S, so ring S-1 is the greedy relay from the last stage to the first.
// A message larger than a slot travels as consecutive slot-sized pieces, so the object's
// size does not grow with n_ctx (S * SHM_SLOTS * SHM_SLOT_BYTES + 4 KiB: 32 MiB at S = 8).
// The sender waits for its stream and copies the device buffer into the next free slot,
// then publishes it; the receiver copies the slot into its device buffer on its stream and
// frees the slot.  One abort word fails every stage's waits.
//
// Life cycle: stage 0 removes any object left under the name (a crashed run), creates a
// fresh one (O_EXCL), reserves its pages (posix_fallocate: a /dev/shm too small fails here
// with an error instead of SIGBUS on the first write), writes the header and only then the
// magic word.  The other stages open the name, wait for the magic, check n_stages and the
// slot size, and join.  Once all S have joined, stage 0 unlinks the name: the mappings stay
// valid, nothing is left in /dev/shm, and a reconnect under the same name starts from a new
// zeroed object.  A stage that mapped a stale object (the name was replaced under it) sees
// the inode change while it waits and reopens.
constexpr int SHM_SLOTS = 4;
constexpr size_t SHM_SLOT_BYTES = (size_t) 1 << 20;
constexpr uint64_t SHM_MAGIC = 0x6c766b73686d3031ull;   // "lvkshm01"
struct ShmRing {
    std::atomic<uint64_t> head;        // pieces published (the sender writes)
    std::atomic<uint64_t> tail;        // pieces consumed (the receiver writes)
    uint64_t bytes[SHM_SLOTS];
};
struct ShmHeader {
    std::atomic<uint64_t> magic;       // SHM_MAGIC once stage 0 has initialised the object
    std::atomic<uint32_t> abort;
    std::atomic<uint32_t> joined;
    uint32_t n_stages;
    uint32_t slots;
    uint64_t slot_bytes;
    std::atomic<uint32_t> go;          // set by stage 0 once all S stages have joined this object
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory rings need address-free atomics");
constexpr size_t SHM_DATA_OFF = 4096;

struct ShmTransport final : StageTransport {
    std::string shm_name;
    int S = 1, stage = 0;
    size_t slot = SHM_SLOT_BYTES, total = 0;
    uint8_t * base = nullptr;
    ShmHeader * h = nullptr;
    bool named = false;                // stage 0: the name still points at our object
    const char * name() const override { return "shm"; }
    ShmRing * ring(int r) const { return (ShmRing *) (base + sizeof(ShmHeader)) + r; }
    uint8_t * data(int r, uint64_t seq) const {
        return base + SHM_DATA_OFF + ((size_t) r * SHM_SLOTS + (size_t) (seq % SHM_SLOTS)) * slot;
    }
    template <class F>
    void spin_until(F ready, const char * what) {
        const double limit = stage_timeout_s();
        const auto t0 = Clock::now();
        for (int i = 0; !ready(); ++i) {
            if (h->abort.load(std::memory_order_acquire))
                throw Error(std::string("llama.vk_amd: stage link aborted by a peer (") + what + ")");
            if (since_s(t0) > limit) {
                abort();
                throw Error(std::string("llama.vk_amd: stage link timed out (") + what + ")");
            }
            if (i > 1024) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    void unmap() {
        if (base) munmap(base, total);
        base = nullptr;
        h = nullptr;
    }
    // stage 0: a fresh object under the name, header written, magic last
    void create() {
        shm_unlink(shm_name.c_str());               // a stale object of a crashed run (ENOENT is fine)
        const int fd = shm_open(shm_name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) throw Error("llama.vk_amd: shm_open(" + shm_name + ", O_EXCL) failed: " + strerror(errno));
        named = true;
        int e = ftruncate(fd, (off_t) total) == 0 ? 0 : errno;
        if (!e) e = posix_fallocate(fd, 0, (off_t) total);
        if (e) {
            close(fd);
            shm_unlink(shm_name.c_str());
            named = false;
            throw Error("llama.vk_amd: the shm link needs " + std::to_string(total >> 20) + " MiB in /dev/shm (" +
                        shm_name + "): " + strerror(e));
        }
        void * p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) throw Error("llama.vk_amd: mmap of the shm link failed");
        base = (uint8_t *) p;
        h = (ShmHeader *) base;
        h->n_stages = (uint32_t) S;
        h->slots = SHM_SLOTS;
        h->slot_bytes = slot;
        h->joined.store(0, std::memory_order_relaxed);
        h->abort.store(0, std::memory_order_relaxed);
        h->go.store(0, std::memory_order_relaxed);
        h->magic.store(SHM_MAGIC, std::memory_order_release);
    }
    // stages 1..S-1: map the object once it exists and is initialised; false = try again
    bool try_open(ino_t & ino) {
        const int fd = shm_open(shm_name.c_str(), O_RDWR, 0600);
        if (fd < 0) return false;
        struct stat sb;
        if (fstat(fd, &sb) != 0 || (size_t) sb.st_size < total) { close(fd); return false; }
        void * p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) return false;
        base = (uint8_t *) p;
        h = (ShmHeader *) base;
        if (h->magic.load(std::memory_order_acquire) != SHM_MAGIC) { unmap(); return false; }
        if (h->n_stages != (uint32_t) S || h->slots != (uint32_t) SHM_SLOTS || h->slot_bytes != slot) {
            unmap();
            throw Error("llama.vk_amd: shm link " + shm_name + " was created for another stage count or slot size");
        }
        ino = sb.st_ino;
        return true;
    }
    // the name now refers to another object (or none) and ours was not completed: stale
    bool replaced(ino_t ino) const {
        struct stat sb;
        const std::string path = "/dev/shm" + shm_name;
        return stat(path.c_str(), &sb) == 0 && sb.st_ino != ino;
    }
    void open_ring(const char * nm, int n_stages, int st) {
        shm_name = nm[0] == '/' ? nm : std::string("/") + nm;
        if (shm_name.find('/', 1) != std::string::npos) throw Error("llama.vk_amd: shm link names may not contain '/'");
        S = n_stages;
        stage = st;
        total = SHM_DATA_OFF + (size_t) S * SHM_SLOTS * slot;
        if (sizeof(ShmHeader) + (size_t) S * sizeof(ShmRing) > SHM_DATA_OFF) throw Error("llama.vk_amd: too many stages for the shm link");
        const double limit = stage_timeout_s();
        const auto t0 = Clock::now();
        if (stage == 0) {
            create();
            h->joined.fetch_add(1, std::memory_order_acq_rel);
            spin_until([&] { return h->joined.load(std::memory_order_acquire) >= (uint32_t) S; }, "joining");
            h->go.store(1, std::memory_order_release);  // the joiners wait for this, not for the count
            shm_unlink(shm_name.c_str());             // every stage has mapped it
            named = false;
            return;
        }
        for (int i = 0;; ++i) {
            ino_t ino = 0;
            if (try_open(ino)) {
                // an object a dead stage 0 left behind may already count S - 1 or more joins:
                // the join completes only when a live stage 0 sets `go`, and a count already at
                // S means the object belonged to a completed (dead) connect
                bool stale = h->joined.fetch_add(1, std::memory_order_acq_rel) >= (uint32_t) S;
                for (int k = 0; !stale && !h->go.load(std::memory_order_acquire); ++k) {
                    if (h->abort.load(std::memory_order_acquire)) throw Error("llama.vk_amd: stage link aborted by a peer (joining)");
                    if (since_s(t0) > limit) { abort(); throw Error("llama.vk_amd: stage link timed out (joining)"); }
                    if ((k & 255) == 255 && replaced(ino)) { stale = true; break; }
                    if (k > 1024) std::this_thread::sleep_for(std::chrono::microseconds(50));
                }
                if (!stale) return;
                unmap();
            }
            if (since_s(t0) > limit) throw Error("llama.vk_amd: stage link timed out waiting for stage 0 to create " + shm_name);
            std::this_thread::sleep_for(std::chrono::microseconds(i < 100 ? 100 : 1000));
        }
    }
    ~ShmTransport() override {
        unmap();
        if (named) shm_unlink(shm_name.c_str());       // stage 0 failed before every stage joined
    }
    void send(const void * d, size_t bytes, int peer, hipStream_t s) override {
        if (peer != (stage + 1) % S) throw Error("llama.vk_amd: bad shm link send");
        ShmRing & r = *ring(stage);
        LVK_HIP(hipStreamSynchronize(s));
        size_t off = 0;
        do {
            const size_t n = std::min(slot, bytes - off);
            const uint64_t seq = r.head.load(std::memory_order_relaxed);
            spin_until([&] { return seq - r.tail.load(std::memory_order_acquire) < (uint64_t) SHM_SLOTS; }, "free slot");
            LVK_HIP(hipMemcpy(data(stage, seq), (const uint8_t *) d + off, n, hipMemcpyDeviceToHost));
            r.bytes[seq % SHM_SLOTS] = n;
            r.head.store(seq + 1, std::memory_order_release);
            off += n;
        } while (off < bytes);
    }
    void recv(void * d, size_t bytes, int peer, hipStream_t s) override {
        if (peer != (stage + S - 1) % S) throw Error("llama.vk_amd: bad shm link recv");
        ShmRing & r = *ring(peer);
        size_t off = 0;
        do {
            const size_t n = std::min(slot, bytes - off);
            const uint64_t seq = r.tail.load(std::memory_order_relaxed);
            spin_until([&] { return r.head.load(std::memory_order_acquire) > seq; }, "message");
            if (r.bytes[seq % SHM_SLOTS] != n) {
                abort();
                throw Error("llama.vk_amd: shm link message size differs between neighbouring stages");
            }
            LVK_HIP(hipMemcpyAsync((uint8_t *) d + off, data(peer, seq), n, hipMemcpyHostToDevice, s));
            LVK_HIP(hipStreamSynchronize(s));     // the slot is reused once tail moves
            r.tail.store(seq + 1, std::memory_order_release);
            off += n;
        } while (off < bytes);
    }
    void wait(hipStream_t s) override { LVK_HIP(hipStreamSynchronize(s)); }
    void abort() noexcept override {
        if (h) h->abort.store(1, std::memory_order_release);
    }
};

}  // namespace

std::unique_ptr<StageTransport> make_rccl_transport(const void * unique_id, int n_stages, int stage, int device) {
    const Rccl & R = Rccl::get();
    ncclUniqueId u;
    std::memcpy(&u, unique_id, sizeof(u));
    std::unique_ptr<RcclTransport> t(new RcclTransport);
    DeviceGuard g(device);
    R.check(R.CommInitRank(&t->comm, n_stages, u, stage), "ncclCommInitRank");
    return t;
}

std::unique_ptr<StageTransport> make_shm_transport(const char * name, int n_stages, int stage) {
    std::unique_ptr<ShmTransport> t(new ShmTransport);
    t->open_ring(name, n_stages, stage);
    return t;
}

double stage_link_probe(Context & c, size_t bytes, int iters) {
    if (!c.link || !c.link->t) throw Error("llama.vk_amd: stage not connected (lvk_stage_connect)");
    StageLink & L = *c.link;
    StageTransport & T = *L.t;
    const int s = L.stage, S = L.n_stages;
    if (S < 2) throw Error("llama.vk_amd: the link probe needs two stages or more");
    if (iters <= 0 || bytes == 0 || bytes > (size_t) c.n_ctx * c.model.hp.n_embd * sizeof(float))
        throw Error("llama.vk_amd: bad link probe size");
    DeviceGuard g(c.device);
    auto lap = [&]() {
        if (s == 0) {
            T.send(c.x, bytes, 1, c.stream);
            T.recv(c.x, bytes, S - 1, c.stream);
        } else {
            T.recv(c.x, bytes, s - 1, c.stream);
            T.send(c.x, bytes, (s + 1) % S, c.stream);
        }
        T.wait(c.stream);
    };
    try {
        for (int i = 0; i < 3; ++i) lap();
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; ++i) lap();
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        return us / iters / S;
    } catch (const Error &) {
        T.abort();
        throw;
    }
}

int stage_step(Context & c, const int * tokens, int n, int n_past, bool greedy, int micro) {
    if (!c.link || !c.link->t) throw Error("llama.vk_amd: stage not connected (lvk_stage_connect)");
    StageLink & L = *c.link;
    StageTransport & T = *L.t;
    const int s = L.stage, S = L.n_stages;
    const size_t E = c.model.hp.n_embd;
    const int V = (int) c.model.hp.n_vocab;
    std::string err;
    DeviceGuard g(c.device);
    try {
        // every argument is checked before the first transfer; a rank that fails anywhere in
        // the step aborts the link, so its neighbours fail instead of waiting on it
        if (greedy && n != 1) throw Error("llama.vk_amd: a greedy stage step takes one token");
        if (n <= 0 || n_past < 0 || n_past + n > c.n_ctx_user) throw Error("llama.vk_amd: n_past + n_tokens exceeds n_ctx");
        if (s == 0) {
            if (!tokens) throw Error("llama.vk_amd: the first stage needs tokens");
            for (int i = 0; i < n; ++i)
                if (tokens[i] < 0 || tokens[i] >= V) throw Error("llama.vk_amd: token id out of range");
        }
        const int m = (micro > 0 && n > micro) ? micro : n;
        for (int off = 0; off < n; off += m) {
            const int k = std::min(m, n - off);
            EvalPart p;
            p.tok_off = off;
            p.n_total = n;
            p.copy_out = off + k == n;
            p.head = p.copy_out || c.logits_all;
            p.greedy = greedy && s == S - 1;
            if (s > 0) T.recv(c.x, (size_t) k * E * sizeof(float), s - 1, c.stream);
            c.begin_eval(s == 0 ? tokens + off : nullptr, k, n_past + off, p);
            if (s + 1 < S) T.send(c.x, (size_t) k * E * sizeof(float), s + 1, c.stream);
        }
        // greedy decode: the last stage's device argmax goes straight to the first stage,
        // whose host needs it to embed the next token
        if (greedy && S > 1) {
            if (s == S - 1) T.send(c.greedy_d, sizeof(int), 0, c.stream);
            if (s == 0) {
                T.recv(c.greedy_d, sizeof(int), S - 1, c.stream);
                LVK_HIP(hipMemcpyAsync(c.greedy_h, c.greedy_d, sizeof(int), hipMemcpyDeviceToHost, c.stream));
            }
        }
        T.wait(c.stream);
    } catch (const Error & e) {
        err = e.msg;
        T.abort();
    }
    try {
        c.end_eval(greedy && s == S - 1);
    } catch (const Error & e) {
        if (err.empty()) err = e.msg;
        T.abort();
    }
    if (!err.empty()) {
        c.logits_valid = false;
        throw Error(err);
    }
    return greedy && (s == 0 || s == S - 1) ? *c.greedy_h : 0;
}

}  // namespace lvk
