// volatile_test.cpp -- ggml_graph_compute must not keep a stale device copy of host bytes
// that change behind the CPU page tables between two calls (tests/test_gpu_ggml_graph.py):
//   pinned  the ggml context's buffer is HIP pinned host memory; between the calls the input
//           is rewritten by a hipMemcpy D2H (a DMA: no CPU store, no soft-dirty bit)
//   shared  the buffer is one view of a memfd mapped twice (MAP_SHARED); between the calls the
//           input is rewritten through the OTHER view (this view's page table never sees it)
//   private the buffer is plain private memory rewritten by the CPU (the tracked case)
//   remap   x's bytes are a read-only private mapping of a file (as llama.cpp maps weights);
//           between the calls that mapping is replaced by one of ANOTHER file at the same
//           address (munmap + mmap MAP_FIXED): same range and permissions, other inode
//   mprotect x's bytes are private anonymous memory, written and then made read-only
//           (mprotect PROT_READ) between the calls
// Each case builds z = x + y, computes it, changes x, computes again and checks z both times.
// usage: volatile_test pinned|shared|private|remap|mprotect   (prints "ok <case>" and exits 0)
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ggml.h"

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } \
    } while (0)

static int check(const ggml_tensor * z, const std::vector<float> & x, const std::vector<float> & y, const char * when) {
    const float * zp = (const float *) z->data;
    for (size_t i = 0; i < x.size(); ++i)
        if (zp[i] != x[i] + y[i]) {
            fprintf(stderr, "%s: z[%zu] = %g, want %g\n", when, i, zp[i], x[i] + y[i]);
            return 1;
        }
    return 0;
}

// a temporary file holding the floats v (unlinked at once; the mapping keeps it alive)
static int temp_file(const std::vector<float> & v) {
    char name[] = "/tmp/lvk_volatile_XXXXXX";
    const int fd = mkstemp(name);
    if (fd < 0) { perror("mkstemp"); exit(2); }
    unlink(name);
    const size_t n = v.size() * 4;
    if (write(fd, v.data(), n) != (ssize_t) n) { perror("write"); exit(2); }
    return fd;
}

int main(int argc, char ** argv) {
    const char * mode = argc > 1 ? argv[1] : "private";
    const size_t mem = 8 << 20;
    const int n = 300000;      // > one page per tensor, several pages
    char * buf = nullptr;
    char * other = nullptr;    // shared: the second view of the same pages
    if (!strcmp(mode, "pinned")) {
        CK(hipHostMalloc((void **) &buf, mem, hipHostMallocDefault));
    } else if (!strcmp(mode, "shared")) {
        const int fd = memfd_create("lvk_volatile_test", 0);
        if (fd < 0 || ftruncate(fd, (off_t) mem) != 0) { perror("memfd"); return 2; }
        buf = (char *) mmap(nullptr, mem, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        other = (char *) mmap(nullptr, mem, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (buf == MAP_FAILED || other == MAP_FAILED) { perror("mmap"); return 2; }
    } else {
        buf = (char *) aligned_alloc(4096, mem);
    }
    ggml_init_params ip = {mem, buf, false};
    ggml_context * ctx = ggml_init(ip);
    ggml_tensor * x = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, n);
    ggml_tensor * y = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, n);
    ggml_tensor * z = ggml_add(ctx, x, y);
    std::vector<float> xv(n), yv(n);
    for (int i = 0; i < n; ++i) { xv[i] = (float) i; yv[i] = 0.5f * (float) (i % 977); }
    const size_t xbytes = ((size_t) n * 4 + 4095) & ~(size_t) 4095;
    if (!strcmp(mode, "remap")) {
        void * p = mmap(nullptr, xbytes, PROT_READ, MAP_PRIVATE, temp_file(xv), 0);
        if (p == MAP_FAILED) { perror("mmap"); return 2; }
        x->data = p;
    } else if (!strcmp(mode, "mprotect")) {
        void * p = mmap(nullptr, xbytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) { perror("mmap"); return 2; }
        x->data = p;
        memcpy(x->data, xv.data(), n * 4);
    } else {
        memcpy(x->data, xv.data(), n * 4);
    }
    memcpy(y->data, yv.data(), n * 4);
    ggml_cgraph g = ggml_build_forward(z);
    ggml_graph_compute(ctx, &g);
    if (check(z, xv, yv, "first call")) return 1;

    // the new x, written past this view's page table
    for (int i = 0; i < n; ++i) xv[i] = -3.0f * (float) i + 1.0f;
    if (!strcmp(mode, "pinned")) {
        float * d = nullptr;
        CK(hipMalloc((void **) &d, n * 4));
        CK(hipMemcpy(d, xv.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(x->data, d, n * 4, hipMemcpyDeviceToHost));   // DMA into the pinned buffer
        CK(hipFree(d));
    } else if (!strcmp(mode, "shared")) {
        memcpy(other + ((char *) x->data - buf), xv.data(), n * 4);
    } else if (!strcmp(mode, "remap")) {
        // another file at the same address, read-only and private like the first
        const int fd = temp_file(xv);
        if (munmap(x->data, xbytes) != 0) { perror("munmap"); return 2; }
        void * p = mmap(x->data, xbytes, PROT_READ, MAP_PRIVATE | MAP_FIXED, fd, 0);
        if (p != x->data) { perror("mmap fixed"); return 2; }
    } else if (!strcmp(mode, "mprotect")) {
        memcpy(x->data, xv.data(), n * 4);
        if (mprotect(x->data, xbytes, PROT_READ) != 0) { perror("mprotect"); return 2; }
    } else {
        memcpy(x->data, xv.data(), n * 4);
    }
    ggml_cgraph g2 = ggml_build_forward(z);
    ggml_graph_compute(ctx, &g2);
    if (check(z, xv, yv, "second call")) return 1;
    ggml_free(ctx);
    printf("ok %s\n", mode);
    return 0;
}
