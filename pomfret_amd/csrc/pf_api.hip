// pf_api.hip -- C ABI of libpomfret_amd.so (declared in include/pomfret_amd.h).
//
// Host driver around the three methphase kernels (pf_kernels.hip):
//   upload  : validate the SoA batch, canonicalise per-read call order, size the
//             HBM workspace, copy everything to the device once (resident batch);
//   launch  : K1 sites -> K2 methmers -> K3 greedy on one HIP stream, then async
//             D2H of the 2x2 tables, site counts and forward tags;
//   finish  : wait, re-run with larger arenas if a device arena overflowed
//             (deterministic: results never depend on arena sizes), then the
//             host epilogue (Fisher test + join decision, pf_host.c).
#include <hip/hip_runtime.h>
#include <mutex>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <thread>
#include <vector>
#include "pf_device.h"
#include "pf_load.h"
#include "pf_host.h"
#include "../../include/pomfret_amd.h"

__global__ void pf_k12_sites_methmers(pf_dev_batch d);
__global__ void pf_k2_methmers(pf_dev_batch d);
__global__ void pf_k12_chunks(pf_dev_batch d);
__global__ void pf_k3_greedy(pf_dev_batch d);
__global__ void pf_k3_wave(pf_dev_batch d);
__global__ void pf_k3_fallback(pf_dev_batch d);
__global__ void pf_k3_heavy(pf_dev_batch d);
__global__ void pf_k3_kdict(pf_dev_batch d);
__global__ void pf_k0_load(pf_load_dev d);
__global__ void pf_k0_multi(pf_load_dev d);
__global__ void pf_k0_scan(pf_load_dev d);
__global__ void pf_k0_pack(pf_load_dev d);
__global__ void pf_k0_pack_small(pf_load_dev d);
__global__ void pf_selftest_div(unsigned long long *bad);
__global__ void pf_selftest_wave(unsigned long long *bad);

#define PF_NKERN 7
#define PF_SLOTS 2
// I/O block header: status u32[4] | arena counters u64[3] (16) | K2, K3
// fallback counters u32 (40, 44) | record level: staging bump pointer u64
// (48), kept reads u32 (56), calls u64 (64), site slots u64 (72) | the heavy
// kernel's deferral counter u32 (80) | the main greedy kernel's problem
// counter u32 (84) | pf_k12_chunks' item count u32 (88) and next item u32 (92) | K0's multi-entry
// record count u32 (96) | pad
#define PF_IO_HDR 128ull

// kernel timing slots: "pf_k0_pack" is the scan + pack pair
static const char *k_names[PF_NKERN] = {"pf_k0_load", "pf_k0_pack", "pf_k12_sites_methmers", "pf_k12_chunks",
                                        "pf_k2_methmers", "pf_k3_wave", "pf_k3_fallback"};
#define PF_GROWABLE (PF_ST_KEYS_OVF | PF_ST_BIG_OVF | PF_ST_SCR_OVF | PF_ST_STAGE_OVF | PF_ST_CALL_OVF | PF_ST_SITES_OVF)

struct pf_ctx {
    int device;
    hipStream_t stream;
    hipStream_t stream2;      /* the heavy greedy problems, beside the main greedy kernel; the fetch's copies */
    hipStream_t stream3;      /* the fetch's second inflate stream (created by the first fetch, so a
                                 context that only runs resident batches keeps two streams: with two
                                 contexts per GPU, four streams for the box's four hardware queues) */
    hipEvent_t ev[PF_NKERN + 1];
    float last_ms[PF_NKERN];
    int have_times;
    float heavy_ms;           /* last run's pf_k3_heavy time (-1: not launched) */
    int k3_block;             /* last run's main greedy kernel: 1 the 256-thread build, 0 the one-wave build */
    float haptag_ms;          /* last pf_haptag_reads kernel time */
    const char *haptag_name;  /* and the kernel that ran */
    int have_haptag;
    void *pin = nullptr;      /* pinned staging for large uploads (grown on demand) */
    size_t pin_cap = 0;
    void *stage = nullptr;    /* pinned staging of the device fetch's compressed bytes */
    size_t stage_cap = 0;
};

// The greedy kernels' dynamic-LDS limits (hipFuncSetAttribute) hold per
// function and device, for every context of the device: kept per device under
// a lock and only ever raised, so one context's smaller batch never lowers the
// limit another context's launch relies on.
static std::mutex g_lds_mu;
static uint32_t g_lds_set[64][4];             // [device][greedy, fallback, one-wave, heavy]
static int raise_lds_limit(int dev, int which, const void *const *fns, int nf, uint32_t need) {
    if (dev < 0 || dev >= 64) return PF_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_lds_mu);
    if (need <= g_lds_set[dev][which]) return PF_OK;
    for (int i = 0; i < nf; i++) {
        const hipError_t e = hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)need);
        if (e != hipSuccess) {
            fprintf(stderr, "[W::pomfret_amd] hipFuncSetAttribute(%u B dynamic LDS): %s\n", need, hipGetErrorString(e));
            (void)hipGetLastError();
            return PF_ERR_HIP;
        }
    }
    g_lds_set[dev][which] = need;
    return PF_OK;
}

struct pf_dbatch {
    pf_ctx *ctx;
    pf_cfg_t cfg;
    uint32_t W, R;
    uint64_t N;
    // host copies used by the epilogue
    std::vector<uint32_t> h_win_read_off;
    std::vector<uint8_t> h_read_hp;
    // device buffers (owned)
    std::vector<void *> allocs;
    pf_dev_batch d;
    // I/O block on the device and its two pinned host slots: launches
    // alternate between the slots, so the host epilogue of one run overlaps
    // the kernels of the next (at most PF_SLOTS runs in flight)
    uint8_t *io = nullptr, *h_io[PF_SLOTS] = {nullptr, nullptr};
    uint64_t io_bytes = 0;
    hipEvent_t ev[PF_SLOTS][PF_NKERN + 1];   // kernel boundaries per slot
    hipEvent_t done[PF_SLOTS];               // slot's D2H complete
    hipEvent_t hev[PF_SLOTS][2];             // pf_k3_heavy's boundaries on the context's second stream
    hipEvent_t fev[PF_SLOTS][2];             // pf_k3_fallback's (after the join with the heavy kernel)
    uint32_t n_heavy = 0;                    // k3_order's first n_heavy problems run in pf_k3_heavy
    std::vector<uint32_t> h_heavy;           // and those problems
    bool heavy_launched[PF_SLOTS] = {false, false};
    int have_ev = 0;
    uint64_t n_launch = 0, n_finish = 0;
    uint64_t site_total;
    // I/O block layout after the header (byte offsets): 2x2 tables, site
    // counts, read counts, then (record level) the window read offsets and
    // each read's record, then the forward tags and (record level) raw tags
    uint64_t o_wro = 0, o_rrec = 0, o_hpfwd = 0, o_hpraw = 0;
    // record-level batches (pf_batch_upload_aln): K0 + scan + pack run first
    // in every launch and size the batch on the device; R is the record count
    // (an upper bound) until a run has finished
    bool has_aln = false;
    uint32_t n_recs = 0;
    bool have_map = false;
    pf_load_dev ld;
    std::vector<uint32_t> h_rec_of_read;
    unsigned long long *k0_ctr = nullptr;
};

// views of one host slot of the I/O block
struct IoView {
    uint32_t *status;
    unsigned long long *ctr;     // keys, big, scr counters after a run
    uint32_t *fb, *k3fb, *k3fbh;
    uint64_t stage, N, sites;    // record level: the staging arena, calls and site slots needed
    uint32_t R;
    int32_t *table;
    uint32_t *S, *nreads;
    uint32_t *wro, *rrec;        // record level: window read offsets, record of each read
    uint8_t *hp_fwd, *hp_raw;
};
static IoView io_view(const pf_dbatch *b, const uint8_t *h) {
    uint8_t *hh = const_cast<uint8_t *>(h);
    const uint64_t W = b->W;
    IoView v;
    v.status = reinterpret_cast<uint32_t *>(hh);
    v.ctr = reinterpret_cast<unsigned long long *>(hh + 16);
    v.fb = reinterpret_cast<uint32_t *>(hh + 40);
    v.k3fb = reinterpret_cast<uint32_t *>(hh + 44);
    v.k3fbh = reinterpret_cast<uint32_t *>(hh + 80);
    memcpy(&v.stage, hh + PF_IO_STAGE, 8);
    memcpy(&v.R, hh + PF_IO_R, 4);
    memcpy(&v.N, hh + PF_IO_N, 8);
    memcpy(&v.sites, hh + PF_IO_SITES, 8);
    v.table = reinterpret_cast<int32_t *>(hh + PF_IO_HDR);
    v.S = reinterpret_cast<uint32_t *>(hh + PF_IO_HDR + 32ull * W);
    v.nreads = reinterpret_cast<uint32_t *>(hh + PF_IO_HDR + 36ull * W);
    v.wro = b->has_aln ? reinterpret_cast<uint32_t *>(hh + b->o_wro) : nullptr;
    v.rrec = b->has_aln ? reinterpret_cast<uint32_t *>(hh + b->o_rrec) : nullptr;
    v.hp_fwd = hh + b->o_hpfwd;
    v.hp_raw = b->has_aln ? hh + b->o_hpraw : nullptr;
    return v;
}
static IoView io_view(const pf_dbatch *b, int slot) { return io_view(b, b->h_io[slot]); }

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "[E::pomfret_amd] %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
    return PF_ERR_HIP; } } while (0)

extern "C" int pf_abi_version(void) { return PF_ABI_VERSION; }

extern "C" int pf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" const char *pf_strerror(int code) {
    switch (code) {
    case PF_OK: return "ok";
    case PF_ERR_ARG: return "invalid argument";
    case PF_ERR_HIP: return "HIP runtime error";
    case PF_ERR_NOMEM: return "out of memory";
    case PF_ERR_UNSUPPORTED: return "unsupported configuration";
    case PF_ERR_LIMIT: return "input exceeds a documented limit";
    case PF_ERR_INTERNAL: return "internal error";
    }
    return "unknown";
}

extern "C" int pf_ctx_create(int device, pf_ctx_t **out) {
    if (!out) return PF_ERR_ARG;
    *out = nullptr;
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(device));
    pf_ctx *c = new pf_ctx();
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->stream2 = nullptr;                             // on first use (pf_ctx_stream2)
    c->stream3 = nullptr;
    c->heavy_ms = -1.0f;
    for (int i = 0; i <= PF_NKERN; i++) HIPCHK(hipEventCreate(&c->ev[i]));
    c->have_times = 0;
    c->have_haptag = 0;
    *out = c;
    return PF_OK;
}

extern "C" int pf_selftest(pf_ctx_t *ctx, uint64_t *mismatches) {
    if (!ctx || !mismatches) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    unsigned long long *d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(*d)));
    int rc = PF_OK;
    unsigned long long h = 0;
    if (hipMemsetAsync(d, 0, sizeof(*d), ctx->stream) != hipSuccess) rc = PF_ERR_HIP;
    if (rc == PF_OK) {
        hipLaunchKernelGGL(pf_selftest_div, dim3(65535), dim3(256), 0, ctx->stream, d);
        hipLaunchKernelGGL(pf_selftest_wave, dim3(1024), dim3(64), 0, ctx->stream, d);
        if (hipGetLastError() != hipSuccess) rc = PF_ERR_HIP;
    }
    if (rc == PF_OK && hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) rc = PF_ERR_HIP;
    if (rc == PF_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = PF_ERR_HIP;
    (void)hipFree(d);
    *mismatches = h;
    return rc;
}

extern "C" int pf_ctx_device(const pf_ctx *c) { return c->device; }
extern "C" hipStream_t pf_ctx_stream(const pf_ctx *c) { return c->stream; }
static std::mutex g_stream3_mu;
// The second stream (the heavy greedy problems, the fetch's copies) is created
// on first use: HIP gives each stream a hardware queue until the device's
// queues (GPU_MAX_HW_QUEUES, 4 here) run out and then shares them, so an idle
// second stream per context would take a queue another context's work needs.
extern "C" hipStream_t pf_ctx_stream2(const pf_ctx *c) {
    pf_ctx *m = const_cast<pf_ctx *>(c);
    std::lock_guard<std::mutex> lk(g_stream3_mu);
    if (!m->stream2) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != m->device) (void)hipSetDevice(m->device);
        if (hipStreamCreateWithFlags(&m->stream2, hipStreamNonBlocking) != hipSuccess) m->stream2 = nullptr;
        if (cur >= 0 && cur != m->device) (void)hipSetDevice(cur);
    }
    return m->stream2 ? m->stream2 : m->stream;
}
extern "C" hipStream_t pf_ctx_stream3(const pf_ctx *c) {
    // created on first use, on the context's device (whatever device the
    // calling thread has current), under a lock: any thread may ask first
    pf_ctx *m = const_cast<pf_ctx *>(c);
    std::lock_guard<std::mutex> lk(g_stream3_mu);
    if (!m->stream3) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != m->device) (void)hipSetDevice(m->device);
        if (hipStreamCreateWithFlags(&m->stream3, hipStreamNonBlocking) != hipSuccess) m->stream3 = nullptr;
        if (cur >= 0 && cur != m->device) (void)hipSetDevice(cur);
    }
    return m->stream3 ? m->stream3 : m->stream;
}

// the context's pinned staging buffer for the device fetch's compressed bytes
// (pf_ingest.hip), grown on demand; the caller owns the context's stream
extern "C" uint8_t *pf_ctx_stage(pf_ctx *c, size_t n) {
    if (c->stage_cap < n) {
        if (c->stage) {
            (void)hipStreamSynchronize(c->stream);
            if (c->stream2) (void)hipStreamSynchronize(c->stream2);
            (void)hipHostFree(c->stage);
        }
        c->stage = nullptr;
        c->stage_cap = 0;
        void *p = nullptr;
        const size_t cap = n + n / 4;
        if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
        c->stage = p;
        c->stage_cap = cap;
    }
    return static_cast<uint8_t *>(c->stage);
}

// release the staging buffer when it grew past `keep` bytes
extern "C" void pf_ctx_stage_trim(pf_ctx *c, size_t keep) {
    if (c->stage && c->stage_cap > keep) {
        (void)hipStreamSynchronize(c->stream);
        if (c->stream2) (void)hipStreamSynchronize(c->stream2);
        (void)hipHostFree(c->stage);
        c->stage = nullptr;
        c->stage_cap = 0;
    }
}

extern "C" void pf_fetch_cache_enable(pf_ctx_t *ctx, int on);
extern "C" void pf_ctx_destroy(pf_ctx_t *c) {
    if (!c) return;
    pf_fetch_cache_enable(c, 0);
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (int i = 0; i <= PF_NKERN; i++) (void)hipEventDestroy(c->ev[i]);
    (void)hipStreamDestroy(c->stream);
    if (c->stream2) {
        (void)hipStreamSynchronize(c->stream2);
        (void)hipStreamDestroy(c->stream2);
    }
    if (c->stream3) {
        (void)hipStreamSynchronize(c->stream3);
        (void)hipStreamDestroy(c->stream3);
    }
    if (c->pin) (void)hipHostFree(c->pin);
    if (c->stage) (void)hipHostFree(c->stage);
    delete c;
}

template <typename T>
static int dev_alloc(pf_dbatch *b, T **p, size_t n) {
    void *q = nullptr;
    // 64 B of slack: kernels may read a whole 16-B group past an array's end
    // (K12's dense pass loads call positions four at a time)
    size_t bytes = std::max<size_t>(n, 1) * sizeof(T) + 64;
    if (hipMalloc(&q, bytes) != hipSuccess) return PF_ERR_NOMEM;
    b->allocs.push_back(q);
    *p = static_cast<T *>(q);
    return PF_OK;
}

template <typename T>
static int dev_put(pf_dbatch *b, T **p, const T *src, size_t n) {
    int rc = dev_alloc(b, p, n);
    if (rc) return rc;
    if (n) HIPCHK(hipMemcpy(*p, src, n * sizeof(T), hipMemcpyHostToDevice));
    return PF_OK;
}

// host-side parallel loop over [0, n): f(lo, hi) per thread (up to 16)
template <typename F>
static void par_for(uint64_t n, F f) {
    unsigned nt = std::thread::hardware_concurrency();
    nt = std::max(1u, std::min(nt, 16u));
    if (n < 4096 || nt == 1) { f(0, n); return; }
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(f, n * t / nt, n * (t + 1) / nt);
    f(0, n / nt);
    for (auto &x : th) x.join();
}

// large host -> device copies go through the context's pinned buffer, two
// 256 MiB halves: fill(buf, lo, hi) writes piece k into one half (parallel
// memcpy or the SEQ repack) while the previous piece's DMA runs from the
// other half (async on the context's stream, one event per half)
template <typename F>
static int pinned_stream(pf_ctx *c, void *dst, size_t bytes, F fill) {
    const size_t half = (size_t)256 << 20;
    const size_t want = 2 * half;
    if (c->pin_cap < want) {
        if (c->pin) (void)hipHostFree(c->pin);
        c->pin = nullptr;
        c->pin_cap = 0;
        if (hipHostMalloc(&c->pin, want, hipHostMallocDefault) != hipSuccess) { c->pin = nullptr; return PF_ERR_NOMEM; }
        c->pin_cap = want;
    }
    hipEvent_t ev[2] = {nullptr, nullptr};
    int rc = PF_OK;
    for (int i = 0; i < 2 && !rc; i++)
        if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) rc = PF_ERR_HIP;
    bool used[2] = {false, false};
    for (size_t o = 0, k = 0; o < bytes && !rc; o += half, k++) {
        const int h = (int)(k & 1);
        uint8_t *buf = (uint8_t *)c->pin + h * half;
        if (used[h] && hipEventSynchronize(ev[h]) != hipSuccess) { rc = PF_ERR_HIP; break; }
        const size_t n = std::min(half, bytes - o);
        fill(buf, (uint64_t)o, (uint64_t)(o + n));
        if (hipMemcpyAsync((uint8_t *)dst + o, buf, n, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
            hipEventRecord(ev[h], c->stream) != hipSuccess) { rc = PF_ERR_HIP; break; }
        used[h] = true;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess && !rc) rc = PF_ERR_HIP;
    for (auto e : ev) if (e) (void)hipEventDestroy(e);
    return rc;
}

static int pinned_put(pf_ctx *c, void *dst, const void *src, size_t bytes) {
    if (bytes < ((size_t)4 << 20)) {
        HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
        return PF_OK;
    }
    const uint8_t *s8 = (const uint8_t *)src;
    return pinned_stream(c, dst, bytes, [&](uint8_t *buf, uint64_t lo, uint64_t hi) {
        par_for(hi - lo, [&](uint64_t a, uint64_t b) { memcpy(buf + a, s8 + lo + a, b - a); });
    });
}

template <typename F>
static int pinned_fill(pf_ctx *c, void *dst, size_t bytes, F fill) {
    return pinned_stream(c, dst, bytes, fill);
}

static void free_arena(pf_dbatch *b, void *p) {
    for (size_t i = 0; i < b->allocs.size(); i++)
        if (b->allocs[i] == p) { (void)hipFree(p); b->allocs.erase(b->allocs.begin() + i); return; }
}

extern "C" void pf_batch_free(pf_dbatch_t *b) {
    if (!b) return;
    (void)hipSetDevice(b->ctx->device);
    (void)hipStreamSynchronize(b->ctx->stream);
    for (void *p : b->allocs) (void)hipFree(p);
    for (int i = 0; i < PF_SLOTS; i++) (void)hipHostFree(b->h_io[i]);
    if (b->have_ev)
        for (int i = 0; i < PF_SLOTS; i++) {
            for (int k = 0; k <= PF_NKERN; k++) (void)hipEventDestroy(b->ev[i][k]);
            (void)hipEventDestroy(b->done[i]);
            for (int k = 0; k < 2; k++) {
                (void)hipEventDestroy(b->hev[i][k]);
                (void)hipEventDestroy(b->fev[i][k]);
            }
        }
    delete b;
}

extern "C" uint32_t pf_batch_n_windows(const pf_dbatch_t *b) { return b ? b->W : 0; }
extern "C" uint32_t pf_batch_n_reads(const pf_dbatch_t *b) { return b ? b->R : 0; }
extern "C" uint64_t pf_batch_n_calls(const pf_dbatch_t *b) { return b ? b->N : 0; }

static int mask_words(int k) { int bits = 2 * k; return bits <= 6 ? 1 : 1 << (bits - 6); }

static int batch_build(pf_dbatch *b, const pf_window_batch_t *in, const uint32_t *first, const uint32_t *last,
                       const uint32_t *cpos, const uint8_t *ccat, const uint64_t *win_calls, pf_dbatch_t **out);

static int check_windows(const pf_cfg_t *cfg, const pf_window_batch_t *in) {
    for (uint32_t w = 0; w < in->n_windows; w++) {
        const uint32_t r0 = in->win_read_off[w], r1 = in->win_read_off[w + 1];
        if (r1 < r0) return PF_ERR_ARG;
        if (r1 - r0 > 65535) return PF_ERR_LIMIT;        // 16-bit per-haplotype counters
        int nc = in->win_n_cand ? in->win_n_cand[w] : cfg->n_cand;
        if (nc <= 1) nc = 2;
        if (nc > PF_MAX_NCAND) return PF_ERR_LIMIT;
    }
    return PF_OK;
}

extern "C" int pf_batch_upload(pf_ctx_t *ctx, const pf_cfg_t *cfg, const pf_window_batch_t *in,
                               pf_dbatch_t **out) {
    if (!ctx || !cfg || !in || !out) return PF_ERR_ARG;
    *out = nullptr;
    if (cfg->k < 1 || cfg->k_span < 0) return PF_ERR_ARG;
    // k <= 15: the reference's limit (2-bit methmer characters in a u32 and
    // `char mmr[16]`, cli.c:243, blockjoin.c:3186-3194, 3403)
    if (cfg->k > 15) return PF_ERR_UNSUPPORTED;
    const uint32_t W = in->n_windows, R = in->n_reads;
    const uint64_t N = in->n_calls;
    if (W && (!in->win_start || !in->win_end || !in->win_read_off)) return PF_ERR_ARG;
    if (R && (!in->read_start || !in->read_end || !in->read_hp || !in->read_call_off)) return PF_ERR_ARG;
    if (N && (!in->call_pos || !in->call_cat)) return PF_ERR_ARG;
    if (W && (in->win_read_off[0] != 0 || in->win_read_off[W] != R)) return PF_ERR_ARG;
    if (R && (in->read_call_off[0] != 0 || in->read_call_off[R] != N)) return PF_ERR_ARG;
    if (!W && R) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(ctx->device));

    pf_dbatch *b = new pf_dbatch();
    b->ctx = ctx;
    b->cfg = *cfg;
    b->W = W; b->R = R; b->N = N;
    b->h_win_read_off.assign(in->win_read_off, in->win_read_off + (W ? W + 1 : 0));
    b->h_read_hp.assign(in->read_hp, in->read_hp + R);
    b->n_launch = b->n_finish = 0;
    auto fail = [&](int rc) { pf_batch_free(b); return rc; };

    // ---- per-window limits (parameter clamps of blockjoin.c:4381-4390 in batch_build)
    {
        const int rc = check_windows(cfg, in);
        if (rc) return fail(rc);
    }

    // ---- reads: first/last call in the caller's order, calls sorted by (pos, cat)
    std::vector<uint32_t> first(R), last(R);
    const uint32_t *cpos = in->call_pos;
    const uint8_t *ccat = in->call_cat;
    std::vector<uint32_t> spos;
    std::vector<uint8_t> scat;
    bool need_sort = false;
    for (uint32_t r = 0; r < R; r++) {
        const uint64_t c0 = in->read_call_off[r], c1 = in->read_call_off[r + 1];
        if (c1 < c0) return fail(PF_ERR_ARG);
        first[r] = c1 > c0 ? cpos[c0] : 0;
        last[r] = c1 > c0 ? cpos[c1 - 1] : 0;
        for (uint64_t c = c0; c < c1; c++) {
            if (cpos[c] >= (1u << 29)) return fail(PF_ERR_LIMIT);  // pos<<3 packing (blockjoin.c:3398)
            if (ccat[c] > 2) return fail(PF_ERR_ARG);
            if (c > c0 && (cpos[c] < cpos[c - 1] || (cpos[c] == cpos[c - 1] && ccat[c] < ccat[c - 1])))
                need_sort = true;
        }
    }
    if (need_sort) {
        spos.assign(cpos, cpos + N);
        scat.assign(ccat, ccat + N);
        std::vector<uint64_t> tmp;
        for (uint32_t r = 0; r < R; r++) {
            const uint64_t c0 = in->read_call_off[r], c1 = in->read_call_off[r + 1];
            tmp.resize(c1 - c0);
            for (uint64_t c = c0; c < c1; c++) tmp[c - c0] = ((uint64_t)cpos[c] << 8) | ccat[c];
            std::sort(tmp.begin(), tmp.end());
            for (uint64_t c = c0; c < c1; c++) {
                spos[c] = (uint32_t)(tmp[c - c0] >> 8);
                scat[c] = (uint8_t)(tmp[c - c0] & 0xff);
            }
        }
        cpos = spos.data();
        ccat = scat.data();
    }

    return batch_build(b, in, first.data(), last.data(), cpos, ccat, nullptr, out);
}

// Allocate and fill the device side of a batch.  Calls level: everything from
// `in`.  Record level (win_calls != NULL): `in` holds the windows' records
// (win_read_off = records per window, which also orders the greedy problems)
// and b->R / b->N are capacities; the read, call and site arrays are only
// allocated -- K0, scan and pack fill them on every run -- and the site
// slots are sized from win_calls, an upper bound of each window's calls.
// The main greedy kernel's largest dynamic LDS that still holds four
// problems per CU (its 128 VGPRs allow four waves per SIMD): a quarter of the
// CU's LDS less the kernel's static LDS.  A workgroup's LDS is granted in
// 1 KB units and a quarter of 160 KB is whole units, so the sum may reach it
// exactly (tools/ubench/lds_occ.hip, profiles/r05/lds_occ.txt); the
// occupancy query does not model the units and over-reports past it.
static uint32_t k3_lds_four(int device) {
    static std::mutex mu;
    static std::vector<std::pair<int, uint32_t>> memo;
    std::lock_guard<std::mutex> lk(mu);
    for (auto &e : memo) if (e.first == device) return e.second;
    hipFuncAttributes fa;
    int per_cu = 0;
    const uint32_t st = hipFuncGetAttributes(&fa, (const void *)pf_k3_greedy) == hipSuccess ? (uint32_t)fa.sharedSizeBytes
                                                                                              : 4096u;
    if (hipDeviceGetAttribute(&per_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) != hipSuccess ||
        per_cu <= 0)
        per_cu = 163840;
    (void)hipGetLastError();
    const uint32_t quarter = ((uint32_t)per_cu / 4u) & ~1023u;
    const uint32_t best = quarter > st + 32768u ? (quarter - st) & ~15u : 36864u;
    memo.push_back({device, best});
    return best;
}

static int batch_build(pf_dbatch *b, const pf_window_batch_t *in, const uint32_t *first, const uint32_t *last,
                       const uint32_t *cpos, const uint8_t *ccat, const uint64_t *win_calls, pf_dbatch_t **out) {
    const pf_cfg_t *cfg = &b->cfg;
    const bool aln = win_calls != nullptr;
    const uint32_t W = b->W, R = b->R;
    const uint64_t N = b->N;
    auto fail = [&](int rc) { pf_batch_free(b); return rc; };
    std::vector<int32_t> par(4ull * W);
    std::vector<uint32_t> read_win(aln ? 0 : R);
    std::vector<uint32_t> site_cap(W);
    std::vector<uint64_t> site_off(W);
    uint64_t site_total = 0;
    for (uint32_t w = 0; w < W; w++) {
        const uint32_t r0 = in->win_read_off[w], r1 = in->win_read_off[w + 1];
        int sel = in->win_cov_sel ? in->win_cov_sel[w] : cfg->cov_for_selection;
        int rt = in->win_cov_rt ? in->win_cov_rt[w] : cfg->cov_for_runtime;
        int nc = in->win_n_cand ? in->win_n_cand[w] : cfg->n_cand;
        if (sel <= 0) sel = 1;
        if (nc <= 1) nc = 2;
        par[4 * w] = sel; par[4 * w + 1] = rt; par[4 * w + 2] = nc; par[4 * w + 3] = 0;
        if (!aln)
            for (uint32_t r = r0; r < r1; r++) read_win[r] = w;
        const uint64_t calls = aln ? win_calls[w] : in->read_call_off[r1] - in->read_call_off[r0];
        // a site needs >= sel meth and >= sel unmeth calls
        const uint64_t cap = calls / (2ull * (uint64_t)sel) + 1;
        site_cap[w] = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFF0ull);
        site_off[w] = site_total;
        site_total += site_cap[w];
    }
    b->site_total = site_total;

    pf_dev_batch &d = b->d;
    memset(&d, 0, sizeof(d));
    d.W = W; d.R = R; d.N = N;
    d.k = cfg->k; d.k_span = cfg->k_span;
    d.hard_cov = cfg->hard_cov > 0 ? cfg->hard_cov : 15;
    // k > 5: per-site hash tables (pf_k3_kdict) instead of 4^k-bit masks;
    // PF_K3_KDICT=1 takes them at any k (tests: the same slots)
    {
        const char *kd = getenv("PF_K3_KDICT");
        d.kdict = cfg->k > 5 || (kd && atoi(kd) == 1) ? 1u : 0u;
    }
    d.mw = d.kdict ? 0 : mask_words(cfg->k);
    int rc = 0;
#define PUT(field, src, n) do { rc = dev_put(b, &field, src, n); if (rc) return fail(rc); } while (0)
#define ALLOC(field, n) do { rc = dev_alloc(b, &field, n); if (rc) return fail(rc); } while (0)
#define PUTA(field, src, n) do { rc = (src) ? dev_put(b, &field, src, n) : dev_alloc(b, &field, n); \
                                 if (rc) return fail(rc); } while (0)
    {
        uint32_t *p; PUT(p, in->win_start, W); d.win_start = p;
        PUT(p, in->win_end, W); d.win_end = p;
        PUTA(p, aln ? nullptr : in->win_read_off, W + 1); d.win_read_off = p;
        int32_t *ip; PUT(ip, par.data(), par.size()); d.win_par = ip;
        uint64_t *up; PUTA(up, aln ? nullptr : site_off.data(), W); d.win_site_off = up;
        PUTA(p, aln ? nullptr : site_cap.data(), W); d.win_site_cap = p;
        PUTA(p, in->read_start, R); d.read_start = p;
        PUTA(p, in->read_end, R); d.read_end = p;
        PUTA(p, first, R); d.read_first = p;
        PUTA(p, last, R); d.read_last = p;
        PUTA(p, aln ? nullptr : read_win.data(), R); d.read_win = p;
        uint8_t *bp; PUTA(bp, in->read_hp, R); d.read_hp = bp;
        PUTA(up, in->read_call_off, R + 1); d.read_call_off = up;
        PUTA(p, cpos, N); d.call_pos = p;
        PUTA(bp, ccat, N); d.call_cat = bp;
        // greedy problems heaviest first (reads per window, direction 1 --
        // the longer chains -- first on ties): the first wave of workgroups
        // spreads the long chains over distinct CUs and pairs them with the
        // short ones dispatched last
        std::vector<uint32_t> ord(2ull * W);
        for (uint32_t i = 0; i < 2 * W; i++) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t c) {
            const uint32_t ra = in->win_read_off[(a >> 1) + 1] - in->win_read_off[a >> 1];
            const uint32_t rc2 = in->win_read_off[(c >> 1) + 1] - in->win_read_off[c >> 1];
            if (ra != rc2) return ra > rc2;
            return (a & 1) > (c & 1);
        });
        PUT(p, ord.data(), ord.size()); d.k3_order = p;
        std::vector<uint32_t> word(W);
        for (uint32_t i = 0; i < W; i++) word[i] = i;
        std::stable_sort(word.begin(), word.end(), [&](uint32_t a, uint32_t c) {
            return in->win_read_off[a + 1] - in->win_read_off[a] > in->win_read_off[c + 1] - in->win_read_off[c];
        });
        PUT(p, word.data(), word.size()); d.k12_order = p;
        // Heavy problems: the windows too large for the main kernel's LDS
        // budget (below), run in pf_k3_heavy on the context's second stream
        // beside the main kernel with a 72 KB budget, so that they start at
        // once instead of being deferred to the fallback kernel after it.
        // Round 3 sent the windows with >= 1.25x the median reads there (the
        // main kernel then ran two 72 KB problems per CU); with round 4's
        // compact layout (the candidate cache reads its per-read fields from
        // HBM) the main kernel's 48 KB fit every window of the 60x gap mix
        // (tools/k3_heavy_prof.py), so the split only takes windows from 2,000
        // reads (1,100 under the 36 KB tier of 30x batches): one kernel, the
        // heaviest problems first.  (A heavy kernel asking for 72 KB beside a
        // main kernel of 48 KB problems waits for free CUs until the main
        // kernel drains: profiles/r04/.)  PF_K3_HEAVY_X: a multiple of the median instead;
        // PF_K3_HEAVY=n forces the n heaviest problems (tests; 0: none).
        if (W) {
            std::vector<uint32_t> rw(W);
            for (uint32_t w = 0; w < W; w++) rw[w] = in->win_read_off[w + 1] - in->win_read_off[w];
            std::nth_element(rw.begin(), rw.begin() + (W * 9) / 10, rw.end());
            const uint32_t p90 = rw[(W * 9) / 10];
            std::nth_element(rw.begin(), rw.begin() + W / 2, rw.end());
            const char *hx = getenv("PF_K3_HEAVY_X");       // tuning: the multiple of the median
            const uint32_t thr = hx ? std::max<uint32_t>(1u, (uint32_t)(atof(hx) * rw[W / 2]))
                                    : (p90 <= 400 ? 1100u : 2000u);
            uint32_t nh = 0;
            while (nh < 2 * W && in->win_read_off[(ord[nh] >> 1) + 1] - in->win_read_off[ord[nh] >> 1] >= thr) nh++;
            const char *hv = getenv("PF_K3_HEAVY");
            if (hv) nh = std::min<uint32_t>((uint32_t)atoi(hv), 2 * W);
            b->n_heavy = nh;
            b->h_heavy.assign(ord.begin(), ord.begin() + nh);
        }
    }
    ALLOC(d.fb_list, std::max<uint32_t>(R, 1));
    ALLOC(d.k12c_list, 2ull * (R / PF_K12C_READS + W + 1));
    ALLOC(d.k3_fb_list, std::max<uint32_t>(4 * W, 1));       // the main kernel's deferrals, then pf_k3_heavy's
    ALLOC(d.k3_ntot, std::max<uint32_t>(2 * W, 1));
    ALLOC(d.k12_path, std::max<uint32_t>(W, 1));
    // one I/O block: the counters zeroed before a run (status, arena
    // counters, fallback counter) followed by everything copied back after it,
    // so a step costs one memset and one D2H copy
    b->o_wro = PF_IO_HDR + 40ull * W;
    b->o_rrec = b->o_wro + (aln ? 4ull * (W + 1) : 0ull);
    b->o_hpfwd = b->o_rrec + (aln ? 4ull * R : 0ull);
    b->o_hpraw = b->o_hpfwd + R;
    b->io_bytes = b->o_hpraw + (aln ? R : 0ull);
    ALLOC(b->io, b->io_bytes);
    d.status = reinterpret_cast<uint32_t *>(b->io);
    {
        unsigned long long *cp = reinterpret_cast<unsigned long long *>(b->io + 16);
        d.keys_ctr = cp; d.big_ctr = cp + 1; d.scr_ctr = cp + 2;
    }
    d.fb_ctr = reinterpret_cast<uint32_t *>(b->io + 40);
    d.k3_fb_ctr = reinterpret_cast<uint32_t *>(b->io + 44);
    d.k3_next = reinterpret_cast<uint32_t *>(b->io + 84);
    d.k12c_ctr = reinterpret_cast<uint32_t *>(b->io + 88);
    d.k12c_next = reinterpret_cast<uint32_t *>(b->io + 92);
    d.table = reinterpret_cast<int32_t *>(b->io + PF_IO_HDR);
    d.win_S = reinterpret_cast<uint32_t *>(b->io + PF_IO_HDR + 32ull * W);
    d.win_nreads = reinterpret_cast<uint32_t *>(b->io + PF_IO_HDR + 36ull * W);
    d.hp_fwd = b->io + b->o_hpfwd;
    ALLOC(d.site_pos, site_total);
    ALLOC(d.st1_pos, site_total);
    ALLOC(d.site_q1, site_total);
    ALLOC(d.len0, site_total);
    ALLOC(d.len1, site_total);
    ALLOC(d.rev_ord, R);
    ALLOC(d.k3_side, 14ull * R + 16);
    ALLOC(d.mmr_n, 2ull * R);
    ALLOC(d.mmr_start, 2ull * R);
    ALLOC(d.mmr_off, 2ull * R);
    ALLOC(d.mmr_cap, R);
    ALLOC(d.big_off, R);
    // arenas: initial sizes; overflow is detected on device and the run repeated
    d.keys_cap = N + (uint64_t)R * (6ull * cfg->k + 8) + 1024;
    ALLOC(d.keys, d.keys_cap);
    d.big_cap = 16ull << 20;
    ALLOC(d.big, d.big_cap);
    d.scr_cap = 64ull << 20;
    ALLOC(d.scr, d.scr_cap);
    ALLOC(d.stats, 16ull * W);
    ALLOC(d.prof, 80ull * W);
    // greedy kernels' dynamic LDS.  40-48 KB (+ ~6 KB static) fits three
    // workgroups per CU, 72 KB two; a problem the main kernel cannot fit runs
    // in the fallback kernel after it.  Small windows (90 % of the windows
    // with <= 400 reads, ~30x) nearly all fit 40 KB, and the higher occupancy
    // pays (30x: K3 2.43 -> 1.95 ms); for larger windows (60x) the heaviest
    // problems would be deferred to a serial tail, so 72 KB
    // (profiles/r02/k3_lds_sweep).  PF_K3_LDS (tests, tuning) sets both.
    // Round 4: the slim loop keeps no per-site divisor cache, u16 per-read
    // fields and, when a window's slot lists miss LDS, only its candidates'
    // lists (k3_greedy_slim CACHE); with the slim kernels' 3.7 KB of static
    // LDS, 48 KB puts three problems on a CU and 36 KB four (LDS is granted
    // in ~1 KB units: 49.5 KB already drops to two, tools/ubench/lds_occ.hip,
    // profiles/r04/lds_occ.txt).  Profiled needs by window reads
    // (tools/k3_heavy_prof.py): on the 60x gap mix every window below 1,284
    // reads fits 44 KB, the largest 49 KB.
    // Round 5: the side arrays of the candidate-cache layout live in HBM
    // (k3_side_mem) and the main kernel fits 128 VGPRs, so at the four-per-CU
    // budget (k3_lds_four, ~37 KB) every problem of the 60x gap mix fits
    // (largest 36.0 KB, at 1,431 reads; tools/k3_heavy_prof.py): four
    // problems per CU when no window passes PF_K3_FOUR_RMAX records (2,000,
    // where the heavy split starts), or when 90 % of the windows are small
    // (the heavy kernel takes the rest).  A problem past the budget takes
    // path 6 (its count table in HBM, k3_run): forced on every problem of the
    // mix it costs 14 % of K3 (4.10 -> 4.68 ms, profiles/r05/ab_k3_path6_forced.txt),
    // so four per CU with every problem on it still matches three per CU
    // without it (4.66 ms); the mix's largest windows hold 1,503-1,514
    // records for at most 1,431 kept reads and all fit the budget.
    uint32_t lds_auto = 49152u;
    if (W) {
        std::vector<uint32_t> rw(W);
        for (uint32_t w = 0; w < W; w++) rw[w] = in->win_read_off[w + 1] - in->win_read_off[w];
        const uint32_t rmax = *std::max_element(rw.begin(), rw.end());
        std::nth_element(rw.begin(), rw.begin() + (W * 9) / 10, rw.end());
        const char *fr = getenv("PF_K3_FOUR_RMAX");
        const uint32_t four_rmax = fr ? (uint32_t)atoi(fr) : 2000u;
        if (rw[(W * 9) / 10] <= 400 || rmax <= four_rmax) lds_auto = k3_lds_four(b->ctx->device);
    }
    const char *lds = getenv("PF_K3_LDS"), *ldf = getenv("PF_K3_LDS_FB"), *ldw = getenv("PF_K3W_LDS");
    // one-wave greedy kernel: ~25 KB leaves six problems per CU (a 60x
    // window's compact image is ~18-23 KB); larger problems go to the fallback
    d.lds_w = ldw ? (uint32_t)atoi(ldw) : 25600u;
    d.lds_bytes = lds ? (uint32_t)atoi(lds) : lds_auto;
    d.lds_fb = ldf ? (uint32_t)atoi(ldf) : lds ? d.lds_bytes : 73728u;
    if (d.lds_fb < d.lds_bytes) d.lds_fb = d.lds_bytes;
    {
        const char *lh = getenv("PF_K3_LDS_HEAVY");
        d.lds_heavy = lh ? (uint32_t)atoi(lh) : d.lds_fb;
        if (d.lds_heavy < d.lds_bytes) d.lds_heavy = d.lds_bytes;
    }
    // PF_K12_CAP / PF_K12_SMAX lower the fused kernel's limits (tests use them
    // to drive reads and windows through the fallback paths)
    const char *kc = getenv("PF_K12_CAP"), *ks = getenv("PF_K12_SMAX");
    d.k12_capw = kc ? std::min<uint32_t>((uint32_t)atoi(kc), PF_K12_CAPW) : PF_K12_CAPW;
    d.k12_smax = ks ? std::min<uint32_t>((uint32_t)atoi(ks), PF_K12_SMAX) : PF_K12_SMAX;
    {
        // windows whose methmer phase K12 hands to pf_k12_chunks: those with
        // at least 900 reads that alone exceed twice a CU's share of the
        // batch's reads (records) -- a window that would be K12's tail.  On a
        // 1024-window 60x batch none qualifies (K12 is throughput-bound
        // there, and the chunks cost 0.1-0.2 ms); alone, the 500 kb window's
        // K12 drops from 1.91 to 0.85 ms (profiles/r05/ab_chunk.txt).
        // PF_K12C_MINR=n forces the bound (0: never).  And the window's
        // sites must fit the kernel's LDS beside its wave buffers.
        const char *km = getenv("PF_K12C_MINR");
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, b->ctx->device) != hipSuccess ||
            ncu <= 0)
            ncu = 256;
        (void)hipGetLastError();
        d.k12c_minr = km ? (uint32_t)atoi(km) : std::max<uint32_t>(900u, (uint32_t)(2ull * R / (uint32_t)ncu));
        if (d.k12c_minr == 0) d.k12c_minr = 0xFFFFFFFFu;
        d.k12c_smax = (uint32_t)((PF_K12C_LDS - PF_K12C_WAVES * PF_K12_WB * PF_K12_CAPW) / 14);
    }
    const char *kd = getenv("PF_K12_DENSE");
    d.k12_dense = kd && atoi(kd) ? 1u : 0u;
    const char *ke = getenv("PF_K2_ENTCAP");
    d.k2_entcap = ke ? std::min<uint32_t>((uint32_t)atoi(ke), PF_K2_ENT_CAP) : PF_K2_ENT_CAP;
    // PF_K3_PATH=fold|rows drives every greedy pick through the sequential
    // fold, or every iteration through the chunked record-row path (tests)
    const char *kp = getenv("PF_K3_PATH");
    d.k3_mode = !kp ? 0u : strcmp(kp, "fold") == 0 ? 1u : strcmp(kp, "rows") == 0 ? 2u : 0u;
    {
        // the greedy loop's slot-list source (pf_kernels.hip k3_run: bit 0
        // allows the candidate cache, a value >= 2 disallows the slot lists in
        // LDS): auto (all lists in LDS when they fit, else the cache, else
        // HBM); tests force the others: "0" no cache, "force" the cache
        // always, "hbm" the HBM lists always
        enum { K3C_NONE = 0u, K3C_AUTO = 1u, K3C_HBM = 2u, K3C_FORCE = 3u };
        const char *kc = getenv("PF_K3_CACHE");
        d.k3_cache = !kc ? K3C_AUTO : !strcmp(kc, "0") ? K3C_NONE : !strcmp(kc, "force") ? K3C_FORCE
                   : !strcmp(kc, "hbm") ? K3C_HBM : K3C_AUTO;
        // path 6 (the candidate cache with the count table in HBM) for every
        // candidate-cache problem with u8 count pairs, not only those past
        // the budget: PF_K3_GCNT=force (tests)
        const char *kg = getenv("PF_K3_GCNT");
        d.k3_gcnt = kg && !strcmp(kg, "force") ? 1u : 0u;
    }
    for (int i = 0; i < PF_SLOTS; i++)
        if (hipHostMalloc((void **)&b->h_io[i], b->io_bytes) != hipSuccess) return fail(PF_ERR_NOMEM);
    for (int i = 0; i < PF_SLOTS; i++) {
        for (int k = 0; k <= PF_NKERN; k++)
            if (hipEventCreate(&b->ev[i][k]) != hipSuccess) return fail(PF_ERR_HIP);
        if (hipEventCreate(&b->done[i]) != hipSuccess) return fail(PF_ERR_HIP);
        for (int k = 0; k < 2; k++)
            if (hipEventCreate(&b->hev[i][k]) != hipSuccess || hipEventCreate(&b->fev[i][k]) != hipSuccess)
                return fail(PF_ERR_HIP);
    }
    b->have_ev = 1;
    *out = b;
    return PF_OK;
#undef PUT
#undef PUTA
#undef ALLOC
}

// ---------------------------------------------------------------------------
// Record-level batches: raw BAM fields resident in HBM, K0 in front of K12.
// aln_build sizes and allocates a batch from the records' lengths and small
// fields (host arrays); `fill` places the large arrays (CIGAR, MM, ML and the
// 16-byte aligned SEQ slices at seq_off) -- copied from host buffers by
// pf_batch_upload_aln, gathered from the inflated BAM stream by the device
// fetch (pf_ingest.hip).
extern "C" int pf_aln_build(pf_ctx_t *ctx, const pf_cfg_t *cfg, const pf_load_cfg_t *lc, const pf_aln_batch_t *a,
                            const pf_aln_fill_t *fill, pf_dbatch_t **out) {
    if (!ctx || !cfg || !lc || !a || !fill || !out) return PF_ERR_ARG;
    *out = nullptr;
    if (cfg->k < 1 || cfg->k_span < 0) return PF_ERR_ARG;
    if (cfg->k > 15) return PF_ERR_UNSUPPORTED;     // as pf_batch_upload
    const uint32_t W = a->n_windows, n = a->n_recs;
    if (W && (!a->win_start || !a->win_end || !a->win_rec_off)) return PF_ERR_ARG;
    if (W && (a->win_rec_off[0] != 0 || a->win_rec_off[W] != n)) return PF_ERR_ARG;
    if (!W && n) return PF_ERR_ARG;
    if (n && (!a->flag || !a->mapq || !a->pos || !a->l_qseq || !a->de || !a->hp || !a->cigar_off || !a->mm_off ||
              !a->ml_off))
        return PF_ERR_ARG;
    for (uint32_t w = 0; w < W; w++)
        if (a->win_rec_off[w + 1] < a->win_rec_off[w]) return PF_ERR_ARG;
    // slice sizes (prefix sums below): 16-byte aligned SEQ slices, HBM trigger
    // slices for records whose bound exceeds K0's LDS list, trigger bounds
    std::vector<uint64_t> seq_off(n + 1), scr_off(n + 1), tbound(n);
    std::vector<int> prc(17, 0);
    par_for(n, [&](uint64_t lo, uint64_t hi) {
        int rc = 0;
        for (uint64_t r = lo; r < hi && !rc; r++) {
            if (a->cigar_off[r + 1] < a->cigar_off[r] || a->mm_off[r + 1] < a->mm_off[r] ||
                a->ml_off[r + 1] < a->ml_off[r]) { rc = PF_ERR_ARG; break; }
            const uint64_t sb = ((uint64_t)a->l_qseq[r] + 1) / 2;
            if (a->mm_off[r + 1] - a->mm_off[r] > 0xFFFFFFF0ull || a->ml_off[r + 1] - a->ml_off[r] > 0xFFFFFFF0ull)
                rc = PF_ERR_LIMIT;
            if (a->l_qseq[r] >= (1u << 24)) rc = PF_ERR_LIMIT;   // K0 packs ranks into 24 bits
            seq_off[r] = (sb + PF_K0_SEQ_ALIGN + PF_K0_SEQ_ALIGN - 1) & ~(uint64_t)(PF_K0_SEQ_ALIGN - 1);
            // trigger lists that may exceed the per-wave LDS list get an HBM slice
            const uint64_t mln = a->ml_off[r + 1] - a->ml_off[r], mlen = a->mm_off[r + 1] - a->mm_off[r];
            const uint64_t bound = mln ? mln : (mlen + 1) / 2;
            scr_off[r] = bound > PF_K0_TCAP ? bound : 0;       // ranks, then triggers in place
            tbound[r] = bound;                                 // >= the record's triggers (and explicit calls)
        }
        if (rc) __atomic_store_n(&prc[rc == PF_ERR_LIMIT ? 1 : 0], 1, __ATOMIC_RELAXED);
    });
    if (prc[0]) return PF_ERR_ARG;
    if (prc[1]) return PF_ERR_LIMIT;
    uint64_t so = 0, sc = 0;
    for (uint32_t r = 0; r < n; r++) {
        const uint64_t x = seq_off[r], y = scr_off[r];
        seq_off[r] = so;
        scr_off[r] = sc;
        so += x;
        sc += y;
    }
    seq_off[n] = so;
    scr_off[n] = sc;
    HIPCHK(hipSetDevice(ctx->device));

    pf_dbatch *b = new pf_dbatch();
    b->ctx = ctx;
    b->cfg = *cfg;
    b->has_aln = true;
    auto fail = [&](int rc) { pf_batch_free(b); return rc; };
    pf_load_dev &ld = b->ld;
    memset(&ld, 0, sizeof(ld));
    ld.n_recs = n;
    ld.min_mapq = (uint32_t)lc->min_mapq;
    ld.min_len = (uint32_t)lc->min_len;
    ld.lo = (uint8_t)lc->qual_lo;
    ld.hi = (uint8_t)lc->qual_hi;
    const char *fs = getenv("PF_K0_PATH");
    ld.force_seq = fs && strcmp(fs, "seq") == 0;
    const char *kd = getenv("PF_K0_DIAG");
    ld.diag = kd ? (uint32_t)atoi(kd) : 0u;
    int rc = 0;
#define PUT(field, src, cnt) do { rc = dev_put(b, &field, src, cnt); if (rc) return fail(rc); } while (0)
#define ALLOC(field, cnt) do { rc = dev_alloc(b, &field, cnt); if (rc) return fail(rc); } while (0)
    {
        uint16_t *p16; PUT(p16, a->flag, n); ld.flag = p16;
        uint8_t *p8; PUT(p8, a->mapq, n); ld.mapq = p8;
        uint32_t *p32; PUT(p32, a->pos, n); ld.pos = p32;
        PUT(p32, a->l_qseq, n); ld.l_qseq = p32;
        float *pf; PUT(pf, a->de, n); ld.de = pf;
        uint64_t *p64; PUT(p64, a->cigar_off, n + 1); ld.cigar_off = p64;
        ALLOC(p32, a->cigar_off[n]); ld.cigar = p32;
        PUT(p64, a->mm_off, n + 1); ld.mm_off = p64;
        ALLOC(p8, a->mm_off[n] + 16); ld.mm = p8;            // padded: K0 stages the text with word loads
        PUT(p64, a->ml_off, n + 1); ld.ml_off = p64;
        ALLOC(p8, a->ml_off[n]); ld.ml = p8;
        PUT(p64, seq_off.data(), n + 1); ld.seq_off = p64;
        PUT(p64, scr_off.data(), n + 1); ld.scr_off = p64;
        ALLOC(p32, sc ? sc : 1); ld.scr = p32;
        ALLOC(p8, so ? so : 1); ld.seq = p8;
        if ((rc = fill->fill(fill->user, ctx, &ld, seq_off.data(), so))) return fail(rc);
        // wave slots in decreasing read length: the long records start first
        // and the four waves of a workgroup finish together
        std::vector<uint32_t> ord(n);
        for (uint32_t r = 0; r < n; r++) ord[r] = r;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return a->l_qseq[x] > a->l_qseq[y]; });
        PUT(p32, ord.data(), n); ld.order = p32;
        PUT(p8, a->hp, n); ld.hp = p8;
        // K0's per-record output
        ALLOC(p32, n); ld.rec_n = p32;
        ALLOC(p32, 8ull * n); ld.rec_out = p32;
        // window of each record, records per window, per-window totals (kept
        // then calls: one memset per run)
        std::vector<uint32_t> rw(n);
        for (uint32_t w = 0; w < W; w++)
            for (uint32_t r = a->win_rec_off[w]; r < a->win_rec_off[w + 1]; r++) rw[r] = w;
        PUT(p32, rw.data(), n); ld.rec_win = p32;
        PUT(p32, a->win_rec_off, W + 1); ld.win_rec_off = p32;
        // pack's workgroups: the windows with the most records first (the
        // long copies start in the first wave of workgroups, not in the tail)
        std::vector<uint32_t> wo(W);
        for (uint32_t w = 0; w < W; w++) wo[w] = w;
        std::stable_sort(wo.begin(), wo.end(), [&](uint32_t x, uint32_t y) {
            return a->win_rec_off[x + 1] - a->win_rec_off[x] > a->win_rec_off[y + 1] - a->win_rec_off[y];
        });
        PUT(p32, wo.data(), W); ld.win_order = p32;
        ALLOC(p32, 2ull * W); ld.win_kept = p32; ld.win_calls = p32 + W;
        ALLOC(p64, W + 1); ld.win_call_off = p64;
        unsigned long long *pc; ALLOC(pc, PF_K0_NCTR); ld.ctr = pc; b->k0_ctr = pc;
        uint32_t *ml_; ALLOC(ml_, std::max<uint32_t>(n, 1)); ld.multi_list = ml_;
        if (hipMemset(pc, 0, PF_K0_NCTR * 8) != hipSuccess) return fail(PF_ERR_HIP);
    }
    // ---- capacities: reads <= records; calls <= the records' trigger bounds
    // (implicit-canonical reads may add more: the arenas grow on overflow)
    std::vector<uint64_t> win_calls(W, 0);
    uint64_t tb_total = 0;
    for (uint32_t w = 0; w < W; w++) {
        for (uint32_t r = a->win_rec_off[w]; r < a->win_rec_off[w + 1]; r++) win_calls[w] += tbound[r];
        tb_total += win_calls[w];
    }
    // static staging slices (the trigger bounds), then a bump-allocated tail
    // for implicit-canonical reads
    std::vector<uint64_t> so_(n + 1, 0);
    for (uint32_t r = 0; r < n; r++) so_[r + 1] = so_[r] + tbound[r];
    uint64_t tail = 65536 + tb_total / 64;
    uint64_t call_cap = tb_total + 4096;
    if (getenv("PF_TEST_TIGHT")) {              // tests: every array starts too small, grows, re-runs
        tail = 16;
        call_cap = 64;
        std::fill(win_calls.begin(), win_calls.end(), 0ull);
        std::fill(so_.begin(), so_.end(), 0ull);        // every record takes the bump path
    }
    ld.stage_cap = so_[n] + tail;
    {
        uint64_t *p64; PUT(p64, so_.data(), n + 1); ld.stage_off = p64;
        uint32_t *p32; ALLOC(p32, ld.stage_cap); ld.stage_pos = p32;
        uint8_t *p8; ALLOC(p8, ld.stage_cap); ld.stage_cat = p8;
        // K0's per-slot record rows (the wave slots' order: longest first)
        std::vector<uint32_t> ordh(n);
        for (uint32_t r = 0; r < n; r++) ordh[r] = r;
        std::stable_sort(ordh.begin(), ordh.end(), [&](uint32_t x, uint32_t y) { return a->l_qseq[x] > a->l_qseq[y]; });
        std::vector<pf_k0_hdr> hdr(std::max<uint32_t>(n, 1));
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t r = ordh[k];
            pf_k0_hdr &h = hdr[k];
            memset(&h, 0, sizeof h);
            h.mm_off = a->mm_off[r]; h.mm_len = (uint32_t)(a->mm_off[r + 1] - a->mm_off[r]);
            h.ml_off = a->ml_off[r]; h.ml_len = (uint32_t)(a->ml_off[r + 1] - a->ml_off[r]);
            h.seq_off = seq_off[r];
            h.cig_off = a->cigar_off[r]; h.ncig = (uint32_t)(a->cigar_off[r + 1] - a->cigar_off[r]);
            h.stage_off = so_[r]; h.stage_len = (uint32_t)(so_[r + 1] - so_[r]);
            h.scr_off = scr_off[r]; h.scr_len = (uint32_t)(scr_off[r + 1] - scr_off[r]);
            h.l_qseq = a->l_qseq[r]; h.pos = a->pos[r]; h.rec = r; h.de = a->de[r];
            h.flag_mapq = (uint32_t)a->flag[r] | ((uint32_t)a->mapq[r] << 16);
        }
        {
            std::vector<uint32_t> slot_of(n);
            for (uint32_t k = 0; k < n; k++) slot_of[ordh[k]] = k;
            for (uint32_t w = 0; w < W; w++)
                for (uint32_t r = a->win_rec_off[w]; r < a->win_rec_off[w + 1]; r++) hdr[slot_of[r]].rec_win = w;
        }
        pf_k0_hdr *ph; PUT(ph, hdr.data(), std::max<uint32_t>(n, 1)); ld.hdr = ph;
    }
    b->W = W; b->R = n; b->N = call_cap;
    b->n_recs = n;
    b->n_launch = b->n_finish = 0;
    pf_window_batch_t in;
    memset(&in, 0, sizeof(in));
    in.n_windows = W; in.n_reads = n; in.n_calls = b->N;
    in.win_start = a->win_start; in.win_end = a->win_end; in.win_read_off = a->win_rec_off;
    in.win_cov_sel = a->win_cov_sel; in.win_cov_rt = a->win_cov_rt; in.win_n_cand = a->win_n_cand;
    rc = check_windows(cfg, &in);                  // records per window bound the reads per window
    if (rc) return fail(rc);
    pf_dbatch_t *res = nullptr;
    rc = batch_build(b, &in, nullptr, nullptr, nullptr, nullptr, win_calls.data(), &res);
    if (rc) return rc;                                      // batch_build freed b
    // scan + pack fill the batch's arrays; K0 shares the batch's status word
    pf_dev_batch &d = b->d;
    ld.n_windows = W;
    ld.status = d.status;
    ld.io = b->io;
    ld.call_cap = b->N;
    ld.sites_cap = b->site_total;
    ld.win_read_off = const_cast<uint32_t *>(d.win_read_off);
    ld.io_win_read_off = reinterpret_cast<uint32_t *>(b->io + b->o_wro);
    ld.win_site_off = const_cast<uint64_t *>(d.win_site_off);
    ld.win_site_cap = const_cast<uint32_t *>(d.win_site_cap);
    ld.win_par = d.win_par;
    ld.read_start = const_cast<uint32_t *>(d.read_start);
    ld.read_end = const_cast<uint32_t *>(d.read_end);
    ld.read_first = const_cast<uint32_t *>(d.read_first);
    ld.read_last = const_cast<uint32_t *>(d.read_last);
    ld.read_win = const_cast<uint32_t *>(d.read_win);
    ld.read_rec = reinterpret_cast<uint32_t *>(b->io + b->o_rrec);
    ld.read_hp = const_cast<uint8_t *>(d.read_hp);
    ld.hp_raw = b->io + b->o_hpraw;
    ld.read_call_off = const_cast<uint64_t *>(d.read_call_off);
    ld.call_pos = const_cast<uint32_t *>(d.call_pos);
    ld.call_cat = const_cast<uint8_t *>(d.call_cat);
    ld.stage_ctr = reinterpret_cast<unsigned long long *>(b->io + PF_IO_STAGE);
    ld.multi_ctr = reinterpret_cast<uint32_t *>(b->io + 96);
    b->N = 0;                                   // calls: known once a run has finished
    *out = res;
    return PF_OK;
#undef PUT
#undef ALLOC
}

// host arrays -> device: the large arrays through the context's pinned
// staging, SEQ repacked into 16-byte aligned, zero-padded slices on the way
// (an odd length's pad nibble cleared too: pf_load.h)
struct HostFill {
    const pf_aln_batch_t *a;
};
static int host_fill(void *user, pf_ctx_t *ctx, pf_load_dev *ld, const uint64_t *seq_off, uint64_t seq_bytes) {
    const pf_aln_batch_t *a = static_cast<HostFill *>(user)->a;
    const uint32_t n = a->n_recs;
    int rc;
    if ((rc = pinned_put(ctx, const_cast<uint32_t *>(ld->cigar), a->cigar, 4ull * a->cigar_off[n]))) return rc;
    if (a->mm_off[n] && (rc = pinned_put(ctx, const_cast<uint8_t *>(ld->mm), a->mm, a->mm_off[n]))) return rc;
    if ((rc = pinned_put(ctx, const_cast<uint8_t *>(ld->ml), a->ml, a->ml_off[n]))) return rc;
    return pinned_fill(ctx, const_cast<uint8_t *>(ld->seq), seq_bytes, [&](uint8_t *buf, uint64_t lo, uint64_t hi) {
        const uint64_t r0 = (uint64_t)(std::upper_bound(seq_off, seq_off + n + 1, lo) - seq_off) - 1;
        uint64_t r1 = r0;
        while (r1 < n && seq_off[r1] < hi) r1++;
        par_for(r1 - r0, [&](uint64_t a0, uint64_t a1) {
            for (uint64_t r = r0 + a0; r < r0 + a1; r++) {
                const uint64_t sb = ((uint64_t)a->l_qseq[r] + 1) / 2;
                const uint64_t x0 = std::max(seq_off[r], lo), x1 = std::min(seq_off[r + 1], hi);
                for (uint64_t x = x0; x < x1;) {               // data part, then the zero pad
                    const uint64_t rel = x - seq_off[r];
                    if (rel < sb) {
                        const uint64_t k = std::min(sb - rel, x1 - x);
                        memcpy(buf + (x - lo), a->seq + a->seq_off[r] + rel, k);
                        if ((a->l_qseq[r] & 1u) && rel + k == sb) buf[x - lo + k - 1] &= 0xF0u;   // the pad nibble
                        x += k;
                    } else {
                        memset(buf + (x - lo), 0, x1 - x);
                        x = x1;
                    }
                }
            }
        });
    });
}

extern "C" int pf_batch_upload_aln(pf_ctx_t *ctx, const pf_cfg_t *cfg, const pf_load_cfg_t *lc,
                                   const pf_aln_batch_t *a, pf_dbatch_t **out) {
    if (!ctx || !cfg || !lc || !a || !out) return PF_ERR_ARG;
    *out = nullptr;
    const uint32_t n = a->n_recs;
    if (n && (!a->cigar_off || !a->cigar || !a->seq_off || !a->seq || !a->mm_off || !a->mm || !a->ml_off ||
              !a->ml || !a->l_qseq || !a->flag))
        return PF_ERR_ARG;
    // host-side checks of what the device fetch guarantees by construction:
    // SEQ long enough for l_qseq, CIGAR query length equal to l_qseq
    std::vector<int> prc(1, 0);
    par_for(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t r = lo; r < hi; r++) {
            if (a->cigar_off[r + 1] < a->cigar_off[r] || a->seq_off[r + 1] < a->seq_off[r]) break;
            const uint64_t sb = ((uint64_t)a->l_qseq[r] + 1) / 2;
            bool bad = a->seq_off[r + 1] - a->seq_off[r] < sb;
            // htslib refuses records whose CIGAR query length differs from l_qseq
            // (bam_read1); K0's walk relies on it to stay inside SEQ
            if (!bad && !(a->flag[r] & 4) && a->l_qseq[r] && a->cigar_off[r + 1] > a->cigar_off[r]) {
                uint64_t ql = 0;
                for (uint64_t c = a->cigar_off[r]; c < a->cigar_off[r + 1]; c++) {
                    const uint32_t op = a->cigar[c] & 15u;
                    if (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) ql += a->cigar[c] >> 4;
                }
                bad = ql != a->l_qseq[r];
            }
            if (bad) { __atomic_store_n(&prc[0], 1, __ATOMIC_RELAXED); break; }
        }
    });
    for (uint32_t r = 0; r < n && !prc[0]; r++)
        if (a->cigar_off[r + 1] < a->cigar_off[r] || a->seq_off[r + 1] < a->seq_off[r]) prc[0] = 1;
    if (prc[0]) return PF_ERR_ARG;
    HostFill hf{a};
    pf_aln_fill_t f{host_fill, &hf};
    return pf_aln_build(ctx, cfg, lc, a, &f, out);
}

extern "C" int pf_batch_read_recs(const pf_dbatch_t *b, uint32_t *rec_of_read, uint32_t n) {
    if (!b || !rec_of_read || n < b->R) return PF_ERR_ARG;
    if (!b->has_aln) {
        for (uint32_t i = 0; i < b->R; i++) rec_of_read[i] = i;
        return PF_OK;
    }
    if (!b->have_map) return PF_ERR_ARG;             // known once a run has finished
    memcpy(rec_of_read, b->h_rec_of_read.data(), 4ull * b->R);
    return PF_OK;
}

// workgroups of pf_k3_greedy the device holds at once with `lds` bytes of
// dynamic LDS (occupancy x CUs; PF_K3_PERSIST caps it, tests)
static uint32_t k3_resident(const pf_ctx *c, uint32_t lds) {
    static std::mutex mu;
    static std::vector<std::pair<uint64_t, uint32_t>> memo;
    const uint64_t key = ((uint64_t)c->device << 32) | lds;
    std::lock_guard<std::mutex> lk(mu);
    for (auto &e : memo) if (e.first == key) return e.second;
    int per = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)pf_k3_greedy, PF_K3S_THREADS, lds) != hipSuccess ||
        per <= 0)
        per = 1;
    // the residency model beside the query (LDS granted in 1 KB units, one
    // wave per SIMD per workgroup, 512 VGPRs per SIMD lane): the larger wins
    // -- a workgroup beyond what the device holds starts when one leaves and
    // finds the problem counter spent, so over-counting costs nothing
    {
        hipFuncAttributes fa;
        int lds_cu = 0;
        if (hipFuncGetAttributes(&fa, (const void *)pf_k3_greedy) == hipSuccess &&
            hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, c->device) == hipSuccess &&
            lds_cu > 0 && fa.numRegs > 0) {
            const uint32_t wg_lds = ((uint32_t)fa.sharedSizeBytes + lds + 1023u) & ~1023u;
            const uint32_t by_lds = wg_lds ? (uint32_t)lds_cu / wg_lds : 8u;
            const uint32_t by_vgpr = std::min<uint32_t>(8u, 512u / (((uint32_t)fa.numRegs + 7u) & ~7u));
            per = std::max<int>(per, (int)std::min(by_lds, by_vgpr));
        }
    }
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || ncu <= 0) ncu = 1;
    (void)hipGetLastError();
    uint32_t n = (uint32_t)per * (uint32_t)ncu;
    const char *e = getenv("PF_K3_PERSIST");
    if (e && atoi(e) > 0) n = std::min<uint32_t>(n, (uint32_t)atoi(e));
    memo.push_back({key, n});
    return n;
}

// enqueue one run of the kernels on the context's stream, timing events and
// results into host slot `slot`.  stages < 3 are debug runs without the D2H:
// 0 stops after the loader (K0, scan, pack), 1 after K12, 2 after K2.
static int enqueue(pf_dbatch *b, int slot, int stages = 3) {
    pf_ctx *c = b->ctx;
    pf_dev_batch &d = b->d;
    hipStream_t st = c->stream;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(b->io, 0, PF_IO_HDR, st));
    if (b->W == 0) { HIPCHK(hipEventRecord(b->done[slot], st)); return PF_OK; }
    // the greedy kernels' dynamic LDS limits (per device, only raised)
    if (d.lds_w > 65536u) {
        const void *f[1] = {(const void *)pf_k3_wave};
        (void)raise_lds_limit(c->device, 2, f, 1, d.lds_w);
    }
    {
        const void *f1[1] = {(const void *)pf_k3_greedy};
        const void *f2[1] = {(const void *)pf_k3_fallback};
        const void *f3[1] = {(const void *)pf_k3_heavy};
        if (raise_lds_limit(c->device, 0, f1, 1, d.lds_bytes) || raise_lds_limit(c->device, 1, f2, 1, d.lds_fb) ||
            raise_lds_limit(c->device, 3, f3, 1, d.lds_heavy))
            return PF_ERR_HIP;
    }
    HIPCHK(hipEventRecord(b->ev[slot][0], st));
    if (b->has_aln) {
        // K0: filters + 5mC extraction of every record into staging slices
        HIPCHK(hipMemsetAsync(b->ld.win_kept, 0, 8ull * b->W, st));
        if (b->ld.n_recs) {
            // one workgroup per four wave slots (round 6 measured persistent
            // grids, slots from a counter or dealt statically: 9.2 / 8.0 ms
            // against 5.7 ms, profiles/r06/ab_k0_persist_*.txt)
            hipLaunchKernelGGL(pf_k0_load, dim3((b->ld.n_recs + PF_K0_WAVES - 1) / PF_K0_WAVES),
                               dim3(PF_K0_WAVES * 64), 0, st, b->ld);
            HIPCHK(hipGetLastError());
            // the records with several C m entries K0 handed over (usually none)
            hipLaunchKernelGGL(pf_k0_multi, dim3(std::min<uint32_t>((b->ld.n_recs + PF_K0_WAVES - 1) / PF_K0_WAVES, 512)),
                               dim3(PF_K0_WAVES * 64), 0, st, b->ld);
            HIPCHK(hipGetLastError());
        }
    }
    HIPCHK(hipEventRecord(b->ev[slot][1], st));
    if (b->has_aln) {
        // window offsets, then the batch's read and call arrays
        hipLaunchKernelGGL(pf_k0_scan, dim3(1), dim3(PF_SCAN_THREADS), 0, st, b->ld);
        HIPCHK(hipGetLastError());
        if (b->W >= PF_PACK_PIPE_MIN) hipLaunchKernelGGL(pf_k0_pack, dim3(b->W), dim3(PF_PACK_THREADS), 0, st, b->ld);
        else hipLaunchKernelGGL(pf_k0_pack_small, dim3(b->W), dim3(PF_PACK_THREADS), 0, st, b->ld);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(b->ev[slot][2], st));
    if (stages < 1) return PF_OK;
    HIPCHK(hipMemsetAsync(d.k12_path, 0, b->W, st));
    hipLaunchKernelGGL(pf_k12_sites_methmers, dim3(b->W), dim3(PF_K1_THREADS), 0, st, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(b->ev[slot][3], st));
    if (stages < 2) return PF_OK;
    // the heavy windows' methmer phase (usually a few windows): persistent,
    // two workgroups per CU over K12's item list
    if (d.k12c_minr != 0xFFFFFFFFu) {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || ncu <= 0)
            ncu = 1;
        const uint32_t gc = std::min<uint32_t>(2u * (uint32_t)ncu, (uint32_t)(b->R / PF_K12C_READS + b->W + 1));
        hipLaunchKernelGGL(pf_k12_chunks, dim3(gc), dim3(PF_K12C_WAVES * 64), PF_K12C_LDS, st, d);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(b->ev[slot][4], st));
    if (stages < 2) return PF_OK;
    // fallback reads only (usually none): a grid-stride kernel over K12's list
    const uint64_t waves = 2ull * b->R;
    const uint32_t g2 = (uint32_t)std::min<uint64_t>((waves + PF_K2_WAVES - 1) / PF_K2_WAVES, 512);
    if (g2) hipLaunchKernelGGL(pf_k2_methmers, dim3(g2), dim3(PF_K2_WAVES * 64), 0, st, d);
    HIPCHK(hipGetLastError());
    // k > 5: the slot dictionaries, one workgroup per problem (timed with K2;
    // not in a stage-limited debug run, whose keys stay keys)
    if (d.kdict && b->W && stages >= 3) {
        hipLaunchKernelGGL(pf_k3_kdict, dim3(2 * b->W), dim3(PF_K3_THREADS), 0, st, d);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(b->ev[slot][5], st));
    if (stages < 3) return PF_OK;
    // main greedy kernel: the 256-thread workgroup build; PF_K3_IMPL=wave runs
    // the one-wavefront build (measured slower on MI355X at 30x-60x: one wave
    // per problem leaves the greedy chain's latencies exposed)
    {
        const char *impl = getenv("PF_K3_IMPL");
        c->k3_block = !(impl && strcmp(impl, "wave") == 0);
    }
    const uint32_t nh = c->k3_block ? b->n_heavy : 0u;
    if (nh) {
        // the heavy problems on the second stream, from the same point (K2 done)
        hipStream_t s2 = pf_ctx_stream2(c);
        HIPCHK(hipStreamWaitEvent(s2, b->ev[slot][5], 0));
        HIPCHK(hipEventRecord(b->hev[slot][0], s2));
        // its own deferral list: a problem beyond its budget runs in a fallback
        // launch right behind it on the same stream, beside the main kernel
        pf_dev_batch dh = d;
        dh.k3_fb_list = d.k3_fb_list + 2ull * b->W;
        dh.k3_fb_ctr = reinterpret_cast<uint32_t *>(b->io + 80);
        hipLaunchKernelGGL(pf_k3_heavy, dim3(nh), dim3(PF_K3H_THREADS), d.lds_heavy, s2, dh);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(pf_k3_fallback, dim3(std::min<uint32_t>(nh, 512)), dim3(PF_K3_THREADS), d.lds_fb,
                           s2, dh);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(b->hev[slot][1], s2));
    }
    if (c->k3_block) {
        // persistent: as many workgroups as fit the device at this LDS budget,
        // each taking the next problem (heaviest first) from a counter -- a
        // free slot on any CU takes the next problem, instead of the problem
        // dispatch order binding workgroups to XCDs round-robin
        pf_dev_batch dl = d;
        dl.k3_order = d.k3_order + nh;
        dl.k3_n = 2 * b->W - nh;
        if (dl.k3_n) {
            const uint32_t g = std::min<uint32_t>(dl.k3_n, k3_resident(c, d.lds_bytes));
            hipLaunchKernelGGL(pf_k3_greedy, dim3(g), dim3(PF_K3S_THREADS), d.lds_bytes, st, dl);
        }
    } else
        hipLaunchKernelGGL(pf_k3_wave, dim3(2 * b->W), dim3(64), d.lds_w, st, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(b->ev[slot][6], st));
    // the main kernel's deferred problems (usually none): a grid-stride kernel over its list
    HIPCHK(hipEventRecord(b->fev[slot][0], st));
    hipLaunchKernelGGL(pf_k3_fallback, dim3(std::min<uint32_t>(2 * b->W, 512)), dim3(PF_K3_THREADS), d.lds_fb,
                       st, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(b->fev[slot][1], st));
    HIPCHK(hipEventRecord(b->ev[slot][7], st));
    if (nh) HIPCHK(hipStreamWaitEvent(st, b->hev[slot][1], 0));   // join: the heavy problems are done
    b->heavy_launched[slot] = nh != 0;
    HIPCHK(hipMemcpyAsync(b->h_io[slot], b->io, b->io_bytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(b->done[slot], st));
    return PF_OK;
}

extern "C" int pf_methphase_launch(pf_ctx_t *ctx, pf_dbatch_t *b) {
    if (!ctx || !b || b->ctx != ctx) return PF_ERR_ARG;
    if (b->n_launch - b->n_finish >= PF_SLOTS) return PF_ERR_ARG;   // finish one first
    const int rc = enqueue(b, (int)(b->n_launch % PF_SLOTS));
    if (rc == PF_OK) b->n_launch++;
    return rc;
}

static int grow(pf_dbatch *b, uint8_t **buf, uint64_t *cap, uint64_t need) {
    free_arena(b, *buf);
    uint64_t ncap = std::max<uint64_t>(need + need / 4 + 1024, *cap * 2);
    void *q = nullptr;
    if (hipMalloc(&q, ncap) != hipSuccess) return PF_ERR_NOMEM;
    b->allocs.push_back(q);
    *buf = (uint8_t *)q;
    *cap = ncap;
    return PF_OK;
}

// replace a typed device array by a larger one (contents are not kept: every
// run rewrites the arrays that grow)
template <typename T>
static int realloc_arr(pf_dbatch *b, T **p, uint64_t n) {
    free_arena(b, (void *)*p);
    *p = nullptr;
    return dev_alloc(b, p, n);
}

// grow what a run found too small (status bits) to what it needed
static int grow_for(pf_dbatch *b, uint32_t stt, const IoView &v) {
    pf_dev_batch &d = b->d;
    pf_load_dev &ld = b->ld;
    int rc = 0;
    if (stt & PF_ST_KEYS_OVF) {
        uint8_t *p = (uint8_t *)d.keys;
        uint64_t capb = d.keys_cap * 4;
        rc = grow(b, &p, &capb, v.ctr[0] * 4);
        d.keys = (uint32_t *)p; d.keys_cap = capb / 4;
    }
    if (!rc && (stt & PF_ST_BIG_OVF)) rc = grow(b, &d.big, &d.big_cap, v.ctr[1]);
    if (!rc && (stt & PF_ST_SCR_OVF)) rc = grow(b, &d.scr, &d.scr_cap, v.ctr[2]);
    if (!rc && (stt & PF_ST_STAGE_OVF)) {
        // v.stage: the bump-allocated tail the run needed, after the static slices
        uint64_t base = 0;
        if (hipMemcpy(&base, ld.stage_off + ld.n_recs, 8, hipMemcpyDeviceToHost) != hipSuccess) return PF_ERR_HIP;
        const uint64_t need = base + v.stage;
        const uint64_t cap = std::max<uint64_t>(need + v.stage / 8 + 4096, ld.stage_cap + (ld.stage_cap - base));
        rc = realloc_arr(b, &ld.stage_pos, cap);
        if (!rc) rc = realloc_arr(b, &ld.stage_cat, cap);
        if (!rc) ld.stage_cap = cap;
    }
    if (!rc && (stt & PF_ST_CALL_OVF)) {
        const uint64_t cap = v.N + v.N / 8 + 4096;
        rc = realloc_arr(b, &ld.call_pos, cap);
        if (!rc) rc = realloc_arr(b, &ld.call_cat, cap);
        if (!rc) { d.call_pos = ld.call_pos; d.call_cat = ld.call_cat; ld.call_cap = cap; }
    }
    if (!rc && (stt & PF_ST_SITES_OVF)) {
        const uint64_t cap = v.sites + v.sites / 8 + 1024;
        rc = realloc_arr(b, &d.site_pos, cap);
        if (!rc) rc = realloc_arr(b, &d.st1_pos, cap);
        if (!rc) rc = realloc_arr(b, &d.site_q1, cap);
        if (!rc) rc = realloc_arr(b, &d.len0, cap);
        if (!rc) rc = realloc_arr(b, &d.len1, cap);
        if (!rc) { b->site_total = cap; ld.sites_cap = cap; }
    }
    return rc;
}

// One finished run's status: 0 done, 1 grown (run it again), < 0 an error.
static int settle_status(pf_dbatch *b, uint32_t stt, const IoView &v, int attempt) {
    if (stt == 0) return 0;
    if (stt & PF_ST_FATAL_CIGAR) return PF_ERR_ARG;   // the reference exits (blockjoin.c:776-779)
    if (stt & PF_ST_POS_LIMIT) return PF_ERR_LIMIT;    // pos<<3 packing (3398)
    if (stt & PF_ST_MM_LIMIT) return PF_ERR_LIMIT;     // > PF_K0_MAXT C m entries in one MM tag
    if (attempt >= 6 || (stt & (PF_ST_INTERNAL | PF_ST_SITE_OVF)) || !(stt & PF_GROWABLE)) {
        fprintf(stderr, "[E::pomfret_amd] device status 0x%x\n", stt);
        return PF_ERR_INTERNAL;
    }
    // an array overflowed: drain the stream (a later run in flight used the
    // same arrays and re-runs itself when finished), grow, re-run
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    const int rc = grow_for(b, stt, v);
    return rc ? rc : 1;
}

// the run's sizes (record level: reads, calls and the read -> record map)
static void note_sizes(pf_dbatch *b, const IoView &v) {
    if (!b->has_aln) return;
    b->R = v.R;
    b->N = v.N;
    if (!b->have_map) {
        b->h_rec_of_read.assign(v.rrec, v.rrec + v.R);
        b->have_map = true;
    }
}

extern "C" int pf_methphase_finish(pf_ctx_t *ctx, pf_dbatch_t *b, pf_window_out_t *out) {
    if (!ctx || !b || !out || b->ctx != ctx || b->n_finish == b->n_launch) return PF_ERR_ARG;
    pf_ctx *c = ctx;
    const int slot = (int)(b->n_finish % PF_SLOTS);
    IoView v;
    b->n_finish++;
    for (int attempt = 0;; attempt++) {
        HIPCHK(hipEventSynchronize(b->done[slot]));
        v = io_view(b, slot);                      // the header's sizes are read here
        if (b->W) {
            for (int i = 0; i < PF_NKERN; i++)
                (void)hipEventElapsedTime(&c->last_ms[i], b->ev[slot][i], b->ev[slot][i + 1]);
            (void)hipEventElapsedTime(&c->last_ms[PF_NKERN - 1], b->fev[slot][0], b->fev[slot][1]);
            c->heavy_ms = -1.0f;
            if (b->heavy_launched[slot]) (void)hipEventElapsedTime(&c->heavy_ms, b->hev[slot][0], b->hev[slot][1]);
            (void)hipGetLastError();               // a failed timing query must not fail a later launch check
            c->have_times = 1;
        }
        const uint32_t stt = b->W ? v.status[0] : 0;
        if (getenv("PF_DEBUG_FALLBACK"))
            fprintf(stderr, "[D::pomfret_amd] status 0x%x, K2 fallback reads %u, K3 deferred problems %u (+%u heavy)\n",
                    stt, *v.fb, *v.k3fb, *v.k3fbh);
        const int s = settle_status(b, stt, v, attempt);
        if (s < 0) return s;
        if (s == 0) break;
        const int rc = enqueue(b, slot);
        if (rc) return rc;
    }
    if (b->W == 0) return PF_OK;
    note_sizes(b, v);
    if (out->win_n_reads)
        for (uint32_t w = 0; w < b->W; w++) out->win_n_reads[w] = v.nreads[w];
    if (b->has_aln) pf_decide_windows(b->W, v.wro, v.S, v.table, v.hp_raw, v.hp_fwd, out);
    else pf_decide_windows(b->W, b->h_win_read_off.data(), v.S, v.table, b->h_read_hp.data(), v.hp_fwd, out);
    return PF_OK;
}

// A synchronous debug run up to `stages` (see enqueue), re-run until no array
// overflows; the header's sizes are noted.
static int run_debug(pf_dbatch *b, int stages) {
    if (b->n_launch != b->n_finish) return PF_ERR_ARG;       // a run is in flight
    std::vector<uint8_t> hdr(PF_IO_HDR);
    for (int attempt = 0;; attempt++) {
        int rc = enqueue(b, 0, stages);
        if (rc) return rc;
        HIPCHK(hipStreamSynchronize(b->ctx->stream));
        if (b->W == 0) return PF_OK;
        HIPCHK(hipMemcpy(hdr.data(), b->io, PF_IO_HDR, hipMemcpyDeviceToHost));
        const IoView v = io_view(b, hdr.data());
        const int s = settle_status(b, v.status[0], v, attempt);
        if (s < 0) return s;
        if (s == 0) {
            if (b->has_aln) {
                b->R = v.R;
                b->N = v.N;
                if (!b->have_map && b->R) {
                    b->h_rec_of_read.resize(b->R);
                    HIPCHK(hipMemcpy(b->h_rec_of_read.data(), b->io + b->o_rrec, 4ull * b->R, hipMemcpyDeviceToHost));
                    b->have_map = true;
                }
                if (!b->R) b->have_map = true;
            }
            return PF_OK;
        }
    }
}

extern "C" int pf_methphase_run(pf_ctx_t *ctx, pf_dbatch_t *b, pf_window_out_t *out) {
    int rc = pf_methphase_launch(ctx, b);
    if (rc) return rc;
    return pf_methphase_finish(ctx, b, out);
}

extern "C" int pf_methphase_windows(int device, const pf_cfg_t *cfg, const pf_window_batch_t *batch,
                                    pf_window_out_t *out) {
    pf_ctx_t *ctx = nullptr;
    int rc = pf_ctx_create(device, &ctx);
    if (rc) return rc;
    pf_dbatch_t *b = nullptr;
    rc = pf_batch_upload(ctx, cfg, batch, &b);
    if (!rc) rc = pf_methphase_run(ctx, b, out);
    pf_batch_free(b);
    pf_ctx_destroy(ctx);
    return rc;
}

// ---- debug / parity entry points: run the first kernels only and copy the
// intermediates (sites of one window; methmers of every read) to the host.
extern "C" int pf_batch_debug_sites(pf_dbatch_t *b, uint32_t w, int dir, uint32_t *real,
                                    uint32_t *starts, uint8_t *lens, uint32_t cap) {
    if (!b || w >= b->W || dir < 0 || dir > 1) return PF_ERR_ARG;
    const int rc = run_debug(b, 1);
    if (rc) return rc;
    uint32_t S = 0;
    HIPCHK(hipMemcpy(&S, b->d.win_S + w, 4, hipMemcpyDeviceToHost));
    uint64_t off = 0;
    HIPCHK(hipMemcpy(&off, b->d.win_site_off + w, 8, hipMemcpyDeviceToHost));
    if (S > cap) return PF_ERR_ARG;
    if (S) {
        HIPCHK(hipMemcpy(real, b->d.site_pos + off, 4ull * S, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(starts, (dir ? b->d.st1_pos : b->d.site_pos) + off, 4ull * S, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(lens, (dir ? b->d.len1 : b->d.len0) + off, S, hipMemcpyDeviceToHost));
    }
    return (int)S;
}

extern "C" int64_t pf_batch_debug_methmers(pf_dbatch_t *b, int dir, uint32_t *mmr_n, uint32_t *mmr_start,
                                           uint32_t *keys, uint64_t cap) {
    if (!b || dir < 0 || dir > 1) return PF_ERR_ARG;
    const int rc = run_debug(b, 2);
    if (rc) return rc;
    std::vector<uint32_t> n(2ull * b->R), s0(2ull * b->R);
    std::vector<uint64_t> off(2ull * b->R);
    if (b->R) {
        HIPCHK(hipMemcpy(n.data(), b->d.mmr_n, 8ull * b->R, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(s0.data(), b->d.mmr_start, 8ull * b->R, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(off.data(), b->d.mmr_off, 16ull * b->R, hipMemcpyDeviceToHost));
    }
    uint64_t tot = 0;
    for (uint32_t r = 0; r < b->R; r++) {
        const uint64_t g = 2ull * r + dir;
        mmr_n[r] = n[g];
        mmr_start[r] = s0[g];
        if (tot + n[g] > cap) return PF_ERR_ARG;
        if (n[g]) HIPCHK(hipMemcpy(keys + tot, b->d.keys + off[g], 4ull * n[g], hipMemcpyDeviceToHost));
        tot += n[g];
    }
    return (int64_t)tot;
}

extern "C" int pf_batch_stats(pf_dbatch_t *b, uint64_t *out, uint64_t n) {
    if (!b || !out || n < 16ull * b->W) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(b->ctx->device));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    if (b->W) HIPCHK(hipMemcpy(out, b->d.stats, 16ull * b->W * sizeof(uint64_t), hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < 2ull * b->W; i++) out[i * 8 + 2] &= (1ull << 56) - 1;   // the path byte: pf_batch_k3_paths
    return PF_OK;
}

extern "C" int pf_batch_k3_paths(pf_dbatch_t *b, uint8_t *out, uint64_t n) {
    if (!b || !out || n < 2ull * b->W) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(b->ctx->device));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    std::vector<uint64_t> st(16ull * b->W + 1);
    if (b->W) HIPCHK(hipMemcpy(st.data(), b->d.stats, 16ull * b->W * sizeof(uint64_t), hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < 2ull * b->W; i++) out[i] = (uint8_t)(st[i * 8 + 2] >> 56);
    return PF_OK;
}

extern "C" int pf_batch_k12_paths(pf_dbatch_t *b, uint8_t *out, uint64_t n) {
    if (!b || !out || n < b->W) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(b->ctx->device));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    if (b->W) HIPCHK(hipMemcpy(out, b->d.k12_path, b->W, hipMemcpyDeviceToHost));
    return PF_OK;
}

extern "C" int pf_batch_k3_budget(const pf_dbatch_t *b, uint32_t *out, uint64_t n) {
    if (!b || !out || n < 4) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(b->ctx->device));
    out[0] = b->d.lds_bytes;
    out[1] = k3_resident(b->ctx, b->d.lds_bytes);
    out[2] = b->d.lds_heavy;
    out[3] = b->n_heavy;
    return PF_OK;
}

extern "C" int pf_batch_heavy(const pf_dbatch_t *b, uint32_t *probs, uint32_t cap) {
    if (!b) return PF_ERR_ARG;
    for (uint32_t i = 0; i < b->n_heavy && i < cap && probs; i++) probs[i] = b->h_heavy[i];
    return (int)b->n_heavy;
}

extern "C" int pf_batch_prof(pf_dbatch_t *b, uint64_t *out, uint64_t n) {
    if (!b || !out || n < 80ull * b->W) return PF_ERR_ARG;
    HIPCHK(hipSetDevice(b->ctx->device));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    if (b->W) HIPCHK(hipMemcpy(out, b->d.prof, 80ull * b->W * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PF_OK;
}

extern "C" void pf_ctx_set_haptag_ms(pf_ctx *c, float ms, const char *name) {
    c->haptag_ms = ms; c->have_haptag = 1; c->haptag_name = name;
}

extern "C" int pf_last_kernel_times(pf_ctx_t *ctx, const char **names, float *ms, int *n) {
    if (!ctx || !n) return PF_ERR_ARG;
    const int hv = ctx->heavy_ms >= 0.0f ? 1 : 0;
    const int tot = PF_NKERN + hv + (ctx->have_haptag ? 1 : 0);
    int m = *n < tot ? *n : tot;
    for (int i = 0; i < m; i++) {
        if (i < PF_NKERN) {
            if (names) names[i] = (i == 5 && ctx->k3_block) ? "pf_k3_greedy" : k_names[i];
            if (ms) ms[i] = ctx->have_times ? ctx->last_ms[i] : -1.0f;
        } else if (i == PF_NKERN && hv) {
            if (names) names[i] = "pf_k3_heavy";
            if (ms) ms[i] = ctx->heavy_ms;
        } else {
            if (names) names[i] = ctx->haptag_name;
            if (ms) ms[i] = ctx->haptag_ms;
        }
    }
    *n = tot;
    return PF_OK;
}

extern "C" int64_t pf_batch_debug_calls(pf_dbatch_t *b, uint64_t *call_off, uint32_t *pos, uint8_t *cat,
                                        uint32_t *first, uint32_t *last, uint64_t cap) {
    if (!b || !call_off || !pos || !cat || !first || !last) return PF_ERR_ARG;
    const int rc = run_debug(b, 0);
    if (rc) return rc;
    if (b->N > cap) return PF_ERR_ARG;
    if (b->R == 0) { call_off[0] = 0; return 0; }
    HIPCHK(hipMemcpy(call_off, b->d.read_call_off, 8ull * (b->R + 1), hipMemcpyDeviceToHost));
    if (b->N) {
        HIPCHK(hipMemcpy(pos, b->d.call_pos, 4ull * b->N, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(cat, b->d.call_cat, b->N, hipMemcpyDeviceToHost));
    }
    if (b->R) {
        HIPCHK(hipMemcpy(first, b->d.read_first, 4ull * b->R, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(last, b->d.read_last, 4ull * b->R, hipMemcpyDeviceToHost));
    }
    return (int64_t)b->N;
}

extern "C" int pf_batch_set_hp(pf_dbatch_t *b, const uint8_t *hp, uint32_t n) {
    if (!b || !b->has_aln || n != b->ld.n_recs || (n && !hp)) return PF_ERR_ARG;
    if (!n) return PF_OK;
    HIPCHK(hipSetDevice(b->ctx->device));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    HIPCHK(hipMemcpy(const_cast<uint8_t *>(b->ld.hp), hp, n, hipMemcpyHostToDevice));
    return PF_OK;
}

extern "C" int pf_batch_debug_recs(pf_dbatch_t *b, uint64_t *sizes, uint16_t *flag, uint8_t *mapq, uint32_t *pos,
                                   uint32_t *l_qseq, float *de, uint8_t *hp, uint64_t *cigar_off, uint32_t *cigar,
                                   uint64_t *seq_off, uint8_t *seq, uint64_t *mm_off, uint8_t *mm, uint64_t *ml_off,
                                   uint8_t *ml) {
    if (!b || !sizes || !b->has_aln) return PF_ERR_ARG;
    const pf_load_dev &ld = b->ld;
    const uint64_t n = ld.n_recs;
    HIPCHK(hipSetDevice(b->ctx->device));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    uint64_t last[4] = {0, 0, 0, 0};
    if (n) {
        HIPCHK(hipMemcpy(&last[0], ld.cigar_off + n, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&last[1], ld.seq_off + n, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&last[2], ld.mm_off + n, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&last[3], ld.ml_off + n, 8, hipMemcpyDeviceToHost));
    }
    sizes[0] = n;
    for (int i = 0; i < 4; i++) sizes[1 + i] = last[i];
    if (!flag) return PF_OK;
    if (!mapq || !pos || !l_qseq || !de || !hp || !cigar_off || !cigar || !seq_off || !seq || !mm_off || !mm ||
        !ml_off || !ml)
        return PF_ERR_ARG;
    if (!n) return PF_OK;
    HIPCHK(hipMemcpy(flag, ld.flag, 2 * n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(mapq, ld.mapq, n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(pos, ld.pos, 4 * n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(l_qseq, ld.l_qseq, 4 * n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(de, ld.de, 4 * n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hp, ld.hp, n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cigar_off, ld.cigar_off, 8 * (n + 1), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(seq_off, ld.seq_off, 8 * (n + 1), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(mm_off, ld.mm_off, 8 * (n + 1), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(ml_off, ld.ml_off, 8 * (n + 1), hipMemcpyDeviceToHost));
    if (last[0]) HIPCHK(hipMemcpy(cigar, ld.cigar, 4 * last[0], hipMemcpyDeviceToHost));
    if (last[1]) HIPCHK(hipMemcpy(seq, ld.seq, last[1], hipMemcpyDeviceToHost));
    if (last[2]) HIPCHK(hipMemcpy(mm, ld.mm, last[2], hipMemcpyDeviceToHost));
    if (last[3]) HIPCHK(hipMemcpy(ml, ld.ml, last[3], hipMemcpyDeviceToHost));
    return PF_OK;
}

extern "C" int pf_batch_load_counters(pf_dbatch_t *b, uint64_t *out, int n) {
    if (!b || !out || n < 8) return PF_ERR_ARG;
    for (int i = 0; i < n; i++) out[i] = 0;
    if (n > PF_K0_NCTR) n = PF_K0_NCTR;
    if (!b->has_aln) return PF_OK;
    HIPCHK(hipSetDevice(b->ctx->device));
    HIPCHK(hipStreamSynchronize(b->ctx->stream));
    HIPCHK(hipMemcpy(out, b->k0_ctr, 8ull * n, hipMemcpyDeviceToHost));
    return PF_OK;
}
