// llama_api.cpp -- the drop-in C API (include/llama.h) over the HIP runtime.
//
// Semantics follow the reference implementation (llama.cpp:1579-1852):
// NULL / non-zero returns on failure with the error printed to stderr, the
// context owns model, KV cache and buffers, logits/embeddings pointers stay
// valid until the next eval, no thread safety.  Tokenizer and sampler are host
// code with the reference's exact tie-breaking (same std::priority_queue /
// std::partial_sort / std::discrete_distribution over std::mt19937).
#include <algorithm>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <csignal>
#include <execinfo.h>
#include <fcntl.h>
#include <queue>
#include <sys/mman.h>
#include <unistd.h>

#include "../../../include/llama.h"
#include "../../../include/lvk_ops.h"
#include "lvk_split.h"

namespace {

// ---------------------------------------------------------------------------
// tokenizer: greedy highest-score bigram merging over UTF-8 characters with
// byte fallback (llama.cpp:1199-1350)
// ---------------------------------------------------------------------------
struct Sym {
    int prev, next;
    const char * text;
    size_t n;
};
struct Bigram {
    int left, right;
    float score;
    size_t size;
};
struct BigramLess {   // max-heap on score, ties: smaller left index first
    bool operator()(const Bigram & a, const Bigram & b) const {
        return a.score < b.score || (a.score == b.score && a.left > b.left);
    }
};

size_t utf8_char_len(char c) {
    static const size_t len[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 3, 4};
    return len[(uint8_t) c >> 4];
}

std::vector<int> tokenize(const lvk::Vocab & vocab, const std::string & text, bool bos) {
    std::vector<int> out;
    if (text.empty()) return out;
    if (bos) out.push_back(1);
    std::vector<Sym> syms;
    for (size_t off = 0; off < text.size();) {
        const size_t n = std::min(text.size() - off, utf8_char_len(text[off]));
        const int idx = (int) syms.size();
        syms.push_back({idx - 1, off + n == text.size() ? -1 : idx + 1, text.data() + off, n});
        off += n;
    }
    std::priority_queue<Bigram, std::vector<Bigram>, BigramLess> pq;
    auto try_add = [&](int l, int r) {
        if (l == -1 || r == -1) return;
        const std::string s(syms[l].text, syms[l].n + syms[r].n);
        auto it = vocab.token_to_id.find(s);
        if (it == vocab.token_to_id.end() || (size_t) it->second >= vocab.id_to_token.size()) return;
        pq.push({l, r, vocab.id_to_token[it->second].score, s.size()});
    };
    for (size_t i = 1; i < syms.size(); ++i) try_add((int) i - 1, (int) i);
    while (!pq.empty()) {
        const Bigram b = pq.top();
        pq.pop();
        Sym & L = syms[b.left];
        Sym & R = syms[b.right];
        if (L.n == 0 || R.n == 0 || L.n + R.n != b.size) continue;   // stale
        L.n += R.n;
        R.n = 0;
        L.next = R.next;
        if (R.next >= 0) syms[R.next].prev = b.left;
        try_add(L.prev, b.left);
        try_add(b.left, L.next);
    }
    for (int i = 0; i != -1; i = syms[i].next) {
        auto it = vocab.token_to_id.find(std::string(syms[i].text, syms[i].n));
        if (it == vocab.token_to_id.end()) {
            for (size_t j = 0; j < syms[i].n; ++j) out.push_back((int) (uint8_t) syms[i].text[j] + 3);
        } else {
            out.push_back(it->second);
        }
    }
    return out;
}

// ---------------------------------------------------------------------------
// sampler (llama.cpp:1352-1459)
// ---------------------------------------------------------------------------
int sample_from_top_k(lvk::Context & c, std::vector<std::pair<float, int>> & cand, float top_p);

int sample_top_p_top_k(lvk::Context & c, const std::vector<int> & last, int top_k, float top_p, float temp,
                       float repeat_penalty) {
    const int n_logits = (int) c.model.hp.n_vocab;
    if (!c.logits_valid || c.logits.size() < (size_t) n_logits) {
        // no eval has left host logits (none yet, a failed eval, or lvk_eval_greedy, which
        // keeps them on the device): nothing to sample from
        fprintf(stderr, "llama_sample_top_p_top_k: no logits (call llama_eval first)\n");
        return -1;
    }
    const float * pl = c.logits.data() + c.logits.size() - n_logits;
    if (temp <= 0) {
        float best = pl[0];
        int id = 0;
        for (int i = 1; i < n_logits; ++i)
            if (pl[i] > best) { best = pl[i]; id = i; }
        return id;
    }
    std::vector<std::pair<float, int>> cand;
    cand.reserve(n_logits);
    const float scale = 1.0f / temp;
    // membership in last_n as a flag per id: the reference's std::find per logit
    // (llama.cpp:1404) costs n_vocab * last_n compares (~2M at 32000 x 64)
    std::vector<uint8_t> in_last((size_t) n_logits, 0);
    for (const int t : last)
        if (t >= 0 && t < n_logits) in_last[(size_t) t] = 1;
    for (int i = 0; i < n_logits; ++i) {
        if (in_last[(size_t) i]) {
            if (pl[i] < 0.0f) cand.emplace_back(pl[i] * scale * repeat_penalty, i);
            else cand.emplace_back(pl[i] * scale / repeat_penalty, i);
        } else {
            cand.emplace_back(pl[i] * scale, i);
        }
    }
    const int k = top_k > 0 ? std::min(top_k, n_logits) : n_logits;
    std::partial_sort(cand.begin(), cand.begin() + k, cand.end(),
                      [](const std::pair<float, int> & a, const std::pair<float, int> & b) { return a.first > b.first; });
    cand.resize(k);
    return sample_from_top_k(c, cand, top_p);
}

// the reference's sampler after sample_top_k (llama.cpp:1419-1456): softmax over the k
// candidates in descending order (expf, double sum), the top-p cut, std::discrete_distribution
// over the context's mt19937
int sample_from_top_k(lvk::Context & c, std::vector<std::pair<float, int>> & cand, float top_p) {
    std::vector<float> probs;
    probs.reserve(cand.size());
    const float maxl = cand[0].first;
    double sum = 0.0;
    for (const auto & kv : cand) {
        const float p = expf(kv.first - maxl);
        probs.push_back(p);
        sum += p;
    }
    for (auto & p : probs) p /= sum;
    if (top_p < 1.0) {
        double cum = 0.0;
        for (int i = 0; i < (int) probs.size(); ++i) {
            cum += probs[i];
            if (cum >= top_p) {
                probs.resize(i + 1);
                cand.resize(i + 1);
                break;
            }
        }
    }
    std::discrete_distribution<> dist(probs.begin(), probs.end());
    return cand[dist(c.rng)].second;
}

void default_progress(float progress, void * ud) {
    unsigned * cur = (unsigned *) ud;
    const unsigned pct = (unsigned) (100 * progress);
    while (pct > *cur) {
        ++*cur;
        fprintf(stderr, ".");
        fflush(stderr);
        if (pct >= 100) fprintf(stderr, "\n");
    }
}

}  // namespace

std::vector<lvk::Context *> llama_context::stages() {
    if (split) return split->st;
    return {&c};
}

extern "C" {

struct llama_context_params llama_context_default_params(void) {
    llama_context_params r;
    r.n_ctx = 512;
    r.n_parts = -1;
    r.seed = 0;
    r.f16_kv = false;
    r.logits_all = false;
    r.vocab_only = false;
    r.use_mmap = true;
    r.use_mlock = false;
    r.embedding = false;
    r.progress_callback = nullptr;
    r.progress_callback_user_data = nullptr;
    return r;
}

bool llama_mmap_supported(void) { return true; }
bool llama_mlock_supported(void) { return true; }

// progress of stage s of S mapped onto one 0..1 sweep
struct StageProgress {
    void (*fn)(float, void *);
    void * ud;
    int s, S;
    static void cb(float p, void * self) {
        const StageProgress * sp = (const StageProgress *) self;
        sp->fn((sp->s + p) / sp->S, sp->ud);
    }
};

// load layers [layer_begin, layer_end) of the file into c on the current HIP device
static void load_stage(lvk::Context & c, const char * path_model, const llama_context_params & params, int layer_begin,
                       int layer_end, void (*progress)(float, void *), void * progress_ud) {
    hipStream_t ls = nullptr;
    if (!params.vocab_only) LVK_HIP(hipStreamCreateWithFlags(&ls, hipStreamNonBlocking));
    struct StreamFree { hipStream_t s; ~StreamFree() { if (s) (void) hipStreamDestroy(s); } } ls_guard{ls};
    lvk::load_model(c.model, path_model, params.vocab_only, ls, progress, progress_ud, layer_begin, layer_end);
    c.model.hp.n_ctx = (uint32_t) params.n_ctx;
    if (!params.vocab_only) c.init(params);
}

// devices: one HIP device per stage (empty: no split, the current device)
static llama_context * init_context(const char * path_model, struct llama_context_params params, int layer_begin,
                                    int layer_end, const std::vector<int> & devices = {},
                                    const char * transport = nullptr, int micro = 64) {
    llama_context * ctx = new llama_context;
    lvk::Context & c = ctx->c;
    c.t_start_us = lvk::now_us();
    if (params.seed <= 0) params.seed = (int) time(nullptr);
    c.rng = std::mt19937(params.seed);
    unsigned cur_pct = 0;
    if (!params.progress_callback) {
        params.progress_callback = default_progress;
        params.progress_callback_user_data = &cur_pct;
    }
    try {
        if (devices.size() < 2 || params.vocab_only) {
            load_stage(c, path_model, params, layer_begin, layer_end, params.progress_callback,
                       params.progress_callback_user_data);
        } else {
            // layer split (lvk_split.h): stages 0..S-2 owned by the Split, S-1 is c
            const int S = (int) devices.size();
            int n_layer = 0;
            {
                lvk::Model probe;
                lvk::load_model(probe, path_model, true, nullptr, nullptr, nullptr);
                n_layer = (int) probe.hp.n_layer;
            }
            if (S > n_layer) throw lvk::Error("more split stages than layers");
            ctx->split.reset(new lvk::Split);
            lvk::Split & sp = *ctx->split;
            sp.devices = devices;
            sp.micro = micro;
            for (int s = 0; s < S; ++s) {
                lvk::DeviceGuard g(devices[s]);
                lvk::Context * sc = &c;
                if (s + 1 < S) {
                    sp.owned.emplace_back(new lvk::Context);
                    sc = sp.owned.back().get();
                }
                const auto lr = lvk::stage_layers(n_layer, S, s);
                StageProgress pr{params.progress_callback, params.progress_callback_user_data, s, S};
                load_stage(*sc, path_model, params, lr.first, lr.second, StageProgress::cb, &pr);
                sp.st.push_back(sc);
            }
            sp.connect(transport);
            fprintf(stderr, "llama_init_from_file: layer split over %d stages (%s hand-off, prompt micro-batch %d)\n",
                    S, sp.rccl ? "RCCL send/recv" : "device copy", sp.micro);
        }
        if (!params.vocab_only) {
            size_t kvb = ctx->split ? ctx->split->kv_bytes() : c.kv_bytes();
            fprintf(stderr, "llama_init_from_file: kv self size  = %7.2f MB\n", kvb / 1024.0 / 1024.0);
        }
    } catch (const lvk::Error & e) {
        fprintf(stderr, "error loading model: %s\n", e.msg.c_str());
        fprintf(stderr, "%s: failed to load model\n", __func__);
        delete ctx;
        return nullptr;
    }
    c.t_load_us = lvk::now_us() - c.t_start_us;
    return ctx;
}

// LVK_SPLIT_DEVICES=0,1,... (one stage per listed HIP device, in layer order; a device may
// repeat) or LVK_SPLIT=S (devices 0..S-1); LVK_SPLIT_TRANSPORT=rccl|copy;
// LVK_SPLIT_MICRO=tokens per prompt micro-batch (0: none)
static std::vector<int> env_split_devices() {
    std::vector<int> d;
    if (const char * e = getenv("LVK_SPLIT_DEVICES")) {
        for (const char * q = e; *q;) {
            char * end = nullptr;
            const long v = strtol(q, &end, 10);
            if (end == q) break;
            d.push_back((int) v);
            q = *end == ',' ? end + 1 : end;
        }
    } else if (const char * e2 = getenv("LVK_SPLIT")) {
        for (int i = 0; i < atoi(e2); ++i) d.push_back(i);
    }
    return d;
}

static int env_split_micro() {
    const char * e = getenv("LVK_SPLIT_MICRO");
    return e ? std::max(0, atoi(e)) : 64;
}

// LVK_SEGV_TRACE=1 (diagnostics): a SIGSEGV / SIGBUS / SIGABRT prints the faulting address
// and the native frames to stderr, then the default action runs (core dump / exit 139, 134)
static void segv_trace(int sig, siginfo_t * si, void *) {
    char buf[96];
    const int n = snprintf(buf, sizeof(buf), "llama.vk_amd: signal %d at address %p; native frames:\n", sig,
                           si ? si->si_addr : nullptr);
    if (n > 0) (void) !write(2, buf, (size_t) n);
    void * fr[64];
    backtrace_symbols_fd(fr, backtrace(fr, 64), 2);
    // the mappings, so unsymbolized frames and the faulting address can be placed
    // (open / read / write only: async-signal-safe)
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        (void) !write(2, "/proc/self/maps:\n", 17);
        char mb[4096];
        for (ssize_t r; (r = read(fd, mb, sizeof(mb))) > 0;) (void) !write(2, mb, (size_t) r);
        close(fd);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
static void maybe_install_segv_trace() {
    static bool done = false;
    if (done || !getenv("LVK_SEGV_TRACE")) return;
    done = true;
    struct sigaction sa {};
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
    sigaction(SIGABRT, &sa, nullptr);
}

struct llama_context * llama_init_from_file(const char * path_model, struct llama_context_params params) {
    maybe_install_segv_trace();
    return init_context(path_model, params, 0, -1, env_split_devices(), getenv("LVK_SPLIT_TRANSPORT"),
                        env_split_micro());
}

struct llama_context * lvk_init_split(const char * path_model, struct llama_context_params params, int n_stages,
                                      const int * devices, const char * transport, int micro) {
    if (n_stages < 1 || !devices || micro < 0) {
        fprintf(stderr, "%s: bad split arguments\n", __func__);
        return nullptr;
    }
    return init_context(path_model, params, 0, -1, std::vector<int>(devices, devices + n_stages), transport, micro);
}

int lvk_split_info(struct llama_context * ctx, int * n_stages, int * rccl, int * micro) {
    const lvk::Split * sp = ctx->split.get();
    if (n_stages) *n_stages = sp ? (int) sp->st.size() : 1;
    if (rccl) *rccl = sp && sp->rccl ? 1 : 0;
    if (micro) *micro = sp ? sp->micro : 0;
    return 0;
}

// ---------------------------------------------------------------------------
// pipeline stages (include/lvk_ops.h)
// ---------------------------------------------------------------------------
struct llama_context * lvk_init_stage(const char * path_model, struct llama_context_params params, int layer_begin,
                                      int layer_end) {
    if (params.vocab_only || layer_begin < 0 || layer_end <= layer_begin) {
        fprintf(stderr, "%s: bad layer range [%d, %d)\n", __func__, layer_begin, layer_end);
        return nullptr;
    }
    return init_context(path_model, params, layer_begin, layer_end);
}

int lvk_stage_eval(struct llama_context * ctx, const llama_token * tokens, int n_tokens, int n_past) {
    try {
        ctx->c.eval(tokens, n_tokens, n_past);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
        return 1;
    }
    return 0;
}

int lvk_stage_get_x(struct llama_context * ctx, void * buf, int n_tokens, int on_device) {
    try { ctx->c.x_copy(buf, n_tokens, false, on_device != 0); }
    catch (const lvk::Error & e) { fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str()); return 1; }
    return 0;
}

int lvk_stage_set_x(struct llama_context * ctx, const void * buf, int n_tokens, int on_device) {
    try { ctx->c.x_copy(const_cast<void *>(buf), n_tokens, true, on_device != 0); }
    catch (const lvk::Error & e) { fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str()); return 1; }
    return 0;
}

int lvk_stage_layers(struct llama_context * ctx, int * layer_begin, int * layer_end) {
    *layer_begin = ctx->c.model.layer_begin;
    *layer_end = ctx->c.model.layer_end;
    return (int) ctx->c.model.hp.n_layer;
}

int lvk_rccl_unique_id(void * id, size_t n) {
    try {
        if (!id || n < sizeof(ncclUniqueId)) throw lvk::Error("id buffer smaller than NCCL_UNIQUE_ID_BYTES");
        const lvk::Rccl & R = lvk::Rccl::get();
        ncclUniqueId u;
        R.check(R.GetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, &u, sizeof(u));
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
        return -1;
    }
    return 0;
}

// the checks every stage link makes before it joins its neighbours
static void check_stage_position(llama_context * ctx, int n_stages, int stage) {
    const lvk::Context & c = ctx->c;
    if (ctx->split || n_stages < 1 || stage < 0 || stage >= n_stages) throw lvk::Error("bad stage link arguments");
    if ((stage == 0) != c.model.has_embed || (stage == n_stages - 1) != c.model.has_head)
        throw lvk::Error("the context's layer range does not match its stage position");
}

int lvk_stage_connect(struct llama_context * ctx, const void * id, int n_stages, int stage) {
    try {
        check_stage_position(ctx, n_stages, stage);
        if (!id) throw lvk::Error("bad stage link arguments");
        ctx->c.link.reset();             // an earlier link of this context (aborted or not) goes first
        std::unique_ptr<lvk::StageLink, lvk::StageLinkDel> L(new lvk::StageLink);
        L->stage = stage;
        L->n_stages = n_stages;
        L->t = lvk::make_rccl_transport(id, n_stages, stage, ctx->c.device);
        ctx->c.link = std::move(L);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
        return -1;
    }
    return 0;
}

int lvk_stage_connect_shm(struct llama_context * ctx, const char * name, int n_stages, int stage) {
    try {
        check_stage_position(ctx, n_stages, stage);
        if (!name || !name[0]) throw lvk::Error("bad stage link arguments");
        lvk::Context & c = ctx->c;
        c.link.reset();                  // an earlier link of this context (aborted or not) goes first
        std::unique_ptr<lvk::StageLink, lvk::StageLinkDel> L(new lvk::StageLink);
        L->stage = stage;
        L->n_stages = n_stages;
        L->t = lvk::make_shm_transport(name, n_stages, stage);
        c.link = std::move(L);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
        return -1;
    }
    return 0;
}

int lvk_stage_step(struct llama_context * ctx, const llama_token * tokens, int n_tokens, int n_past, int greedy,
                   int micro) {
    try {
        return lvk::stage_step(ctx->c, tokens, n_tokens, n_past, greedy != 0, micro);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
        return -1;
    }
}

int lvk_stage_link_probe(struct llama_context * ctx, int bytes, int iters, double * us_per_hop) {
    try {
        if (bytes <= 0 || !us_per_hop) throw lvk::Error("llama.vk_amd: bad link probe arguments");
        *us_per_hop = lvk::stage_link_probe(ctx->c, (size_t) bytes, iters);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
        return -1;
    }
    return 0;
}

void llama_free(struct llama_context * ctx) { delete ctx; }

int llama_eval(struct llama_context * ctx, const llama_token * tokens, int n_tokens, int n_past, int n_threads) {
    (void) n_threads;   // host thread count hint; the forward pass runs on the GPU
    lvk::Context & c = ctx->c;
    const int64_t t0 = lvk::now_us();
    try {
        if (ctx->split) ctx->split->eval(tokens, n_tokens, n_past);
        else c.eval(tokens, n_tokens, n_past);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: failed to eval: %s\n", __func__, e.msg.c_str());
        return 1;
    }
    const int64_t dt = lvk::now_us() - t0;
    if (n_tokens == 1) { c.t_eval_us += dt; c.n_eval++; }          // llama.cpp:1186-1195
    else if (n_tokens > 1) { c.t_p_eval_us += dt; c.n_p_eval += n_tokens; }
    if (!c.has_evaluated_once) {
        c.t_load_us = lvk::now_us() - c.t_start_us;
        c.has_evaluated_once = true;
    }
    return 0;
}

int llama_tokenize(struct llama_context * ctx, const char * text, llama_token * tokens, int n_max_tokens,
                   bool add_bos) {
    const std::vector<int> res = tokenize(ctx->c.model.vocab, text, add_bos);
    if (n_max_tokens < (int) res.size()) {
        fprintf(stderr, "%s: too many tokens\n", __func__);
        return -((int) res.size());
    }
    for (size_t i = 0; i < res.size(); ++i) tokens[i] = res[i];
    return (int) res.size();
}

int llama_n_vocab(struct llama_context * ctx) { return (int) ctx->c.model.vocab.id_to_token.size(); }
int llama_n_ctx(struct llama_context * ctx) { return (int) ctx->c.model.hp.n_ctx; }
int llama_n_embd(struct llama_context * ctx) { return (int) ctx->c.model.hp.n_embd; }
float * llama_get_logits(struct llama_context * ctx) { return ctx->c.logits.data(); }
float * llama_get_embeddings(struct llama_context * ctx) { return ctx->c.embedding.data(); }

const char * llama_token_to_str(struct llama_context * ctx, llama_token token) {
    if (token < 0 || token >= llama_n_vocab(ctx)) return nullptr;   // llama.cpp:1761-1766 checks the upper bound only
    return ctx->c.model.vocab.id_to_token[token].text.c_str();
}

llama_token llama_token_bos(void) { return 1; }
llama_token llama_token_eos(void) { return 2; }

llama_token llama_sample_top_p_top_k(struct llama_context * ctx, const llama_token * last_n_tokens_data,
                                     int last_n_tokens_size, int top_k, float top_p, float temp,
                                     float repeat_penalty) {
    lvk::Context & c = ctx->c;
    const int64_t t0 = lvk::now_us();
    const std::vector<int> last(last_n_tokens_data, last_n_tokens_data + last_n_tokens_size);
    const int r = sample_top_p_top_k(c, last, top_k, top_p, temp, repeat_penalty);
    c.t_sample_us += lvk::now_us() - t0;
    c.n_sample++;
    return r;
}

// lvk_eval_sample (include/lvk_ops.h): llama_eval of one token + llama_sample_top_p_top_k,
// the O(n_vocab) part of the sampler on the device (sample.hip)
int lvk_eval_sample(struct llama_context * ctx, int token, int n_past, const int * last_n, int n_last, int top_k,
                    float top_p, float temp, float repeat_penalty) {
    lvk::Context & c = ctx->c;
    if (temp <= 0) return lvk_eval_greedy(ctx, token, n_past);   // llama.cpp:1382-1394
    if (n_last < 0 || (n_last > 0 && !last_n)) {
        fprintf(stderr, "%s: bad last-n window\n", __func__);
        return -1;
    }
    const int n_vocab = (int) c.model.hp.n_vocab;
    const int k = top_k > 0 ? std::min(top_k, n_vocab) : n_vocab;
    auto host_path = [&]() -> int {
        if (llama_eval(ctx, &token, 1, n_past, 1) != 0) return -1;
        return llama_sample_top_p_top_k(ctx, last_n, n_last, top_k, top_p, temp, repeat_penalty);
    };
    if (ctx->split || c.logits_all || k > lvk::SAMPLE_CAP || n_last > lvk::SAMPLE_MAX_LAST || n_vocab > lvk::SAMPLE_MAX_VOCAB)
        return host_path();
    int64_t t0 = lvk::now_us();
    lvk::SampleParams & sp = *c.samp_h;
    sp.k = k;
    sp.n_last = n_last;
    sp.scale = 1.0f / temp;            // llama.cpp:1398
    sp.rp = repeat_penalty;
    if (n_last > 0) std::memcpy(sp.last, last_n, sizeof(int) * (size_t) n_last);
    try {
        c.eval_sample(token, n_past);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: failed to eval: %s\n", __func__, e.msg.c_str());
        return -1;
    }
    c.t_eval_us += lvk::now_us() - t0;
    c.n_eval++;
    t0 = lvk::now_us();
    const lvk::SampleOut & so = *c.sout_h;
    std::vector<std::pair<float, int>> cand;
    bool exact = so.flags == 0 && so.count >= k && so.count <= lvk::SAMPLE_CAP;
    if (exact) {
        cand.reserve((size_t) so.count);
        for (int i = 0; i < so.count; ++i) cand.emplace_back(so.val[i], so.id[i]);
        std::sort(cand.begin(), cand.end(),
                  [](const std::pair<float, int> & a, const std::pair<float, int> & b) { return a.first > b.first; });
        // distinct values: the descending order is the one std::partial_sort leaves; a tie
        // anywhere among the candidates (their order is the heap's) takes the reference path
        for (size_t i = 1; i < cand.size() && exact; ++i) exact = cand[i - 1].first != cand[i].first;
    }
    int r;
    if (exact) {
        cand.resize((size_t) k);
        r = sample_from_top_k(c, cand, top_p);
    } else {
        try {
            c.fetch_logits();
        } catch (const lvk::Error & e) {
            fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
            return -1;
        }
        const std::vector<int> last(last_n, last_n + n_last);
        r = sample_top_p_top_k(c, last, top_k, top_p, temp, repeat_penalty);
        c.n_sample_fallback++;
    }
    c.t_sample_us += lvk::now_us() - t0;
    c.n_sample++;
    return r;
}

const uint8_t * llama_get_kv_cache(struct llama_context * ctx) {
    try {
        if (ctx->split) ctx->split->kv_get(ctx->c.kv_host);
        else ctx->c.kv_get();
    } catch (const lvk::Error & e) { fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str()); }
    return ctx->c.kv_host.data();
}
size_t llama_get_kv_cache_size(struct llama_context * ctx) {
    return ctx->split ? ctx->split->kv_bytes() : ctx->c.kv_bytes();
}
int llama_get_kv_cache_token_count(struct llama_context * ctx) { return ctx->c.kv_n; }
void llama_set_kv_cache(struct llama_context * ctx, const uint8_t * kv_cache, size_t n_size, int n_token_count) {
    if (n_size != llama_get_kv_cache_size(ctx)) {   // LLAMA_ASSERT in the reference (llama.cpp:1696)
        fprintf(stderr, "llama_set_kv_cache: size mismatch\n");
        abort();
    }
    try {
        if (ctx->split) ctx->split->kv_set(kv_cache, n_size);
        else ctx->c.kv_set(kv_cache, n_size);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
    }
    ctx->c.kv_n = n_token_count;
}

void llama_print_timings(struct llama_context * ctx) {
    lvk::Context & c = ctx->c;
    const int64_t t_end = lvk::now_us();
    const int n_sample = std::max(1, c.n_sample), n_eval = std::max(1, c.n_eval), n_p_eval = std::max(1, c.n_p_eval);
    fprintf(stderr, "\n");
    fprintf(stderr, "%s:        load time = %8.2f ms\n", __func__, c.t_load_us / 1000.0);
    fprintf(stderr, "%s:      sample time = %8.2f ms / %5d runs   (%8.2f ms per run)\n", __func__, 1e-3 * c.t_sample_us,
            n_sample, 1e-3 * c.t_sample_us / n_sample);
    fprintf(stderr, "%s: prompt eval time = %8.2f ms / %5d tokens (%8.2f ms per token)\n", __func__,
            1e-3 * c.t_p_eval_us, n_p_eval, 1e-3 * c.t_p_eval_us / n_p_eval);
    fprintf(stderr, "%s:        eval time = %8.2f ms / %5d runs   (%8.2f ms per run)\n", __func__, 1e-3 * c.t_eval_us,
            n_eval, 1e-3 * c.t_eval_us / n_eval);
    fprintf(stderr, "%s:       total time = %8.2f ms\n", __func__, (t_end - c.t_start_us) / 1000.0);
}

void llama_reset_timings(struct llama_context * ctx) {
    lvk::Context & c = ctx->c;
    c.t_start_us = lvk::now_us();
    c.t_sample_us = c.n_sample = 0;
    c.t_eval_us = c.n_eval = 0;
    c.t_p_eval_us = c.n_p_eval = 0;
}

const char * llama_print_system_info(void) {
    static std::string s;
    int dev = 0, n = 0;
    hipDeviceProp_t prop{};
    if (hipGetDeviceCount(&n) == hipSuccess && n > 0 && hipGetDevice(&dev) == hipSuccess)
        (void) hipGetDeviceProperties(&prop, dev);
    s = "HIP = 1 | GPU = ";
    s += n > 0 ? prop.gcnArchName : "none";
    s += " | CUs = " + std::to_string(n > 0 ? prop.multiProcessorCount : 0);
    s += " | HBM = " + std::to_string(n > 0 ? (long long) (prop.totalGlobalMem >> 20) : 0) + " MiB";
    s += " | WAVE64 = 1 | DOT8_I4 = 1 | KV = f16 | ";
    return s.c_str();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// include/llama_internal.h: the model file's tensors by name (reference llama.cpp:1850-1852)
// ---------------------------------------------------------------------------
#include <fcntl.h>

#include "../../../include/llama_internal.h"

namespace {
struct TensorMap {
    void * addr = nullptr;
    size_t size = 0;
    std::vector<ggml_tensor> tensors;
    std::vector<std::pair<std::string, ggml_tensor *>> by_name;
    ~TensorMap() {
        if (addr && size) munmap(addr, size);
    }
};
}  // namespace

std::vector<std::pair<std::string, struct ggml_tensor *>> & llama_internal_get_tensor_map(struct llama_context * ctx) {
    static std::vector<std::pair<std::string, struct ggml_tensor *>> empty;
    if (ctx->tensor_map) return static_cast<TensorMap *>(ctx->tensor_map.get())->by_name;
    try {
        const lvk::Model & m = ctx->c.model;
        size_t fsize = 0;
        const std::vector<lvk::FileTensor> list = lvk::file_tensor_list(m.path, fsize);
        std::shared_ptr<TensorMap> tm = std::make_shared<TensorMap>();
        const int fd = open(m.path.c_str(), O_RDONLY);
        if (fd < 0) throw lvk::Error("cannot open " + m.path);
        tm->addr = mmap(nullptr, fsize, PROT_READ, MAP_SHARED, fd, 0);
        close(fd);
        if (tm->addr == MAP_FAILED) {
            tm->addr = nullptr;
            throw lvk::Error("mmap failed for " + m.path);
        }
        tm->size = fsize;
        tm->tensors.resize(list.size());
        for (size_t i = 0; i < list.size(); ++i) {
            const lvk::FileTensor & f = list[i];
            ggml_tensor & t = tm->tensors[i];
            std::memset(&t, 0, sizeof t);
            // ggjt type ids 0 f32, 1 f16, 2 q4_0, 3 q4_1 (llama.cpp:387-395) -> enum ggml_type
            t.type = f.type == 0 ? GGML_TYPE_F32 : f.type == 1 ? GGML_TYPE_F16 : f.type == 2 ? GGML_TYPE_Q4_0 : GGML_TYPE_Q4_1;
            t.n_dims = (int) f.ne.size();
            for (int d = 0; d < GGML_MAX_DIMS; ++d) t.ne[d] = d < t.n_dims ? f.ne[d] : 1;
            t.nb[0] = ggml_type_size(t.type);
            t.nb[1] = t.nb[0] * (t.ne[0] / ggml_blck_size(t.type));
            for (int d = 2; d < GGML_MAX_DIMS; ++d) t.nb[d] = t.nb[d - 1] * t.ne[d - 1];
            t.op = GGML_OP_NONE;
            t.data = (char *) tm->addr + f.off;
            tm->by_name.emplace_back(f.name, &t);
        }
        ctx->tensor_map = tm;
        return tm->by_name;
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: %s\n", __func__, e.msg.c_str());
        empty.clear();
        return empty;
    }
}
