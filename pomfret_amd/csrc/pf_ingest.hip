// pf_ingest.hip -- host side of the device BAM ingest: BGZF block tables and
// the device inflate entry points (kernels in pf_inflate.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include "pf_ingest.h"
#include "../../include/pomfret_amd.h"

struct pf_ctx;
extern "C" int pf_ctx_device(const pf_ctx *c);
extern "C" hipStream_t pf_ctx_stream(const pf_ctx *c);
extern "C" hipStream_t pf_ctx_stream2(const pf_ctx *c);
extern "C" hipStream_t pf_ctx_stream3(const pf_ctx *c);
extern "C" uint8_t *pf_ctx_stage(pf_ctx *c, size_t n);
extern "C" void pf_ctx_stage_trim(pf_ctx *c, size_t keep);

#define ICHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "[E::pomfret_amd] %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
    rc = PF_ERR_HIP; goto out; } } while (0)

static uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static uint32_t rd32(const uint8_t *p) { return rd16(p) | (rd16(p + 2) << 16); }

// Parse the BGZF blocks of comp[0, len) (whole blocks, as bgzf_read_block
// reads them: gzip member with FEXTRA and the BC subfield) into a block table
// whose outputs are laid out back to back from out_base.  Returns the number
// of blocks, or a negative PF_ERR.
int64_t pf_bgzf_scan(const uint8_t *comp, uint64_t len, uint64_t out_base, uint32_t run,
                     std::vector<pf_bgzf_blk> &blk) {
    uint64_t o = 0, out = out_base;
    int64_t n = 0;
    while (o < len) {
        if (len - o < 18) return PF_ERR_ARG;
        const uint8_t *h = comp + o;
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return PF_ERR_ARG;
        const uint32_t xlen = rd16(h + 10);
        if (12ull + xlen > len - o) return PF_ERR_ARG;
        uint32_t bsize = 0;
        for (uint32_t x = 0; x + 4 <= xlen;) {
            const uint8_t *sf = h + 12 + x;
            const uint32_t slen = rd16(sf + 2);
            if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) bsize = rd16(sf + 4) + 1;
            x += 4 + slen;
        }
        if (bsize < 12 + xlen + 8 || bsize > 65536 || bsize > len - o) return PF_ERR_ARG;
        pf_bgzf_blk b;
        b.in_off = o + 12 + xlen;
        b.in_len = bsize - 12 - xlen - 8;
        b.crc = rd32(h + bsize - 8);
        b.isize = rd32(h + bsize - 4);
        if (b.isize > 65536) return PF_ERR_ARG;
        b.out_off = out;
        b.run = run;
        out += b.isize;
        blk.push_back(b);
        n++;
        o += bsize;
    }
    return n;
}

// Inflate blocks on the device: d_in / d_blk / d_arena / d_status resident;
// status words set per block.  One wavefront per block (pf_inflate).  A
// two-pass decoder (one lane per block for the Huffman decode, then the LZ77
// copies) was built and measured slower; it lives in tools/ubench.
int pf_inflate_launch(pf_ctx *ctx, hipStream_t st, const uint8_t *d_in, const pf_bgzf_blk *d_blk,
                      const pf_bgzf_blk *h_blk, uint32_t nblk, uint8_t *d_arena, uint32_t *d_status, hipEvent_t e0,
                      hipEvent_t e1) {
    (void)ctx;
    (void)h_blk;
    if (e0 && hipEventRecord(e0, st) != hipSuccess) return PF_ERR_HIP;
    if (!nblk) return e1 && hipEventRecord(e1, st) != hipSuccess ? PF_ERR_HIP : PF_OK;   // (the pair stays timeable)
    hipLaunchKernelGGL(pf_inflate, dim3((nblk + 3) / 4), dim3(256), 0, st, d_in, d_blk, nblk, d_arena, d_status);
    if (hipGetLastError() != hipSuccess) return PF_ERR_HIP;
    if (e1 && hipEventRecord(e1, st) != hipSuccess) return PF_ERR_HIP;
    return PF_OK;
}

extern "C" int pf_bgzf_inflate(pf_ctx_t *ctx, const uint8_t *comp, uint64_t comp_len, uint8_t *out, uint64_t out_cap,
                               uint64_t *out_len, uint32_t *block_status, uint32_t status_cap, float *kernel_ms) {
    if (!ctx || (!comp && comp_len) || !out_len) return PF_ERR_ARG;
    std::vector<pf_bgzf_blk> blk;
    const int64_t nb = pf_bgzf_scan(comp, comp_len, 0, 0, blk);
    if (nb < 0) return (int)nb;
    const uint64_t total = blk.empty() ? 0 : blk.back().out_off + blk.back().isize;
    *out_len = total;
    if (total > out_cap || (total && !out)) return PF_ERR_ARG;
    if (!nb) return PF_OK;
    int rc = PF_OK;
    uint8_t *d_in = nullptr, *d_arena = nullptr;
    pf_bgzf_blk *d_blk = nullptr;
    uint32_t *d_st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::vector<uint32_t> st((size_t)nb);
    hipStream_t s = pf_ctx_stream((const pf_ctx *)ctx);
    ICHK(hipSetDevice(pf_ctx_device((const pf_ctx *)ctx)));
    ICHK(hipMalloc(&d_in, comp_len + 512));
    ICHK(hipMemsetAsync(d_in + comp_len, 0, 512, s));
    ICHK(hipMemcpyAsync(d_in, comp, comp_len, hipMemcpyHostToDevice, s));
    ICHK(hipMalloc(&d_blk, sizeof(pf_bgzf_blk) * (size_t)nb));
    ICHK(hipMemcpyAsync(d_blk, blk.data(), sizeof(pf_bgzf_blk) * (size_t)nb, hipMemcpyHostToDevice, s));
    ICHK(hipMalloc(&d_arena, total + 256));
    ICHK(hipMalloc(&d_st, 4ull * (size_t)nb));
    ICHK(hipMemsetAsync(d_st, 0, 4ull * (size_t)nb, s));
    ICHK(hipEventCreate(&e0));
    ICHK(hipEventCreate(&e1));
    rc = pf_inflate_launch((pf_ctx *)ctx, s, d_in, d_blk, blk.data(), (uint32_t)nb, d_arena, d_st, e0, e1);
    if (rc) goto out;
    ICHK(hipMemcpyAsync(st.data(), d_st, 4ull * (size_t)nb, hipMemcpyDeviceToHost, s));
    ICHK(hipMemcpyAsync(out, d_arena, total, hipMemcpyDeviceToHost, s));
    ICHK(hipStreamSynchronize(s));
    if (kernel_ms) ICHK(hipEventElapsedTime(kernel_ms, e0, e1));
    for (int64_t i = 0; i < nb; i++) {
        if (block_status && (uint64_t)i < status_cap) block_status[i] = st[i];
        if (st[i] && rc == PF_OK) rc = PF_ERR_ARG;
    }
out:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d_in);
    (void)hipFree(d_blk);
    (void)hipFree(d_arena);
    (void)hipFree(d_st);
    return rc;
}

// ===========================================================================
// Device fetch: the windows' records from the BAM file through the device
// (inflate, chain, decode, select, gather) into a record-level batch.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <map>
#include <thread>
#include <string>
#include <errno.h>
#include <fcntl.h>
#include <unistd.h>
#include <sys/stat.h>
#include "pf_load.h"

namespace {

struct DevBuf {                                  // device allocations freed together, after the streams drain
    std::vector<void *> p;
    hipStream_t st = nullptr, st2 = nullptr, st3 = nullptr;
    ~DevBuf() {
        if (st2) (void)hipStreamSynchronize(st2);
        if (st3) (void)hipStreamSynchronize(st3);
        if (st) (void)hipStreamSynchronize(st);
        for (void *x : p) (void)hipFree(x);
    }
    template <typename T> T *alloc(size_t n) {
        void *x = nullptr;
        if (hipMalloc(&x, n ? n * sizeof(T) : 1) != hipSuccess) return nullptr;
        p.push_back(x);
        return static_cast<T *>(x);
    }
};

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// one merged byte range of the file and the blocks scanned in it
struct Range {
    uint64_t f0, f1;          // requested [f0, f1) file bytes
    uint64_t buf0;            // its bytes in the compressed upload buffer
    uint64_t end_addr;        // file address after its last whole block
    uint32_t b0, b1;          // its blocks
    bool to_eof;
    uint64_t scan = 0;        // bytes of the run scanned into blocks so far
};

struct Plan {
    std::vector<pf_bgzf_blk> blk;
    std::vector<uint64_t> caddr;            // file address of each block
    std::vector<uint32_t> bsize;            // its BGZF size
    std::vector<Range> runs;
    uint64_t comp_n = 0;                    // compressed bytes of every run, back to back (d_comp), + pad
    uint64_t arena = 0;                     // inflated bytes
};

// Contig arenas kept on the device between the -u pre-pass and the window
// jobs (HBM holds a contig's inflated BAM many times over): the pre-pass
// fetches each contig whole -- a chromosome-scale contig in position pieces of
// about 4 GiB of compressed BAM, each kept as an arena of its own (round 5) --
// and a window job of that contig on the same device then takes its blocks
// from the kept arena whose position range holds every window of the job
// (the driver cuts jobs at the pieces' bounds and places the bounds between
// windows) instead of reading and inflating them again.  Keyed by context,
// file (path, size, mtime), contig and position range; kept while the device
// keeps a reserve free; released by pf_fetch_cache_clear (end of a methphase
// run, context destruction).
struct ArenaCache {
    int64_t pbeg = 0, pend = INT64_MAX;     // the piece's fetch region [pbeg, pend) of the contig
    const pf_ctx_t *ctx = nullptr;
    std::string path;
    uint64_t fsize = 0;
    int64_t mt_s = 0, mt_ns = 0;
    int32_t tid = -1;
    uint8_t *d_arena = nullptr;             // arena bytes + 512 zero bytes
    uint64_t arena = 0;
    std::vector<uint64_t> caddr, out_off;   // per block: file address, arena offset
    std::vector<uint32_t> bsize, isize, run; // its BGZF and inflated sizes, its run
    std::vector<uint64_t> run_f1;           // per run: the end of the file range its scan covered
};
std::mutex g_cache_mu;
std::vector<ArenaCache *> g_cache;
std::map<int, uint64_t> g_kept_dev;         // bytes of kept arenas per device (PF_ARENA_KEEP_MAX)

// PF_ARENA_KEEP_MAX (bytes; K/M/G suffixes): at most this many bytes of kept
// arenas per device -- a smaller HBM, to measure the window jobs' re-reads of
// the contigs past the budget (tools/genome_scale.py).  Unset: no cap beyond
// the free-memory reserve.
uint64_t arena_keep_max() {
    const char *e = getenv("PF_ARENA_KEEP_MAX");
    if (!e || !*e) return UINT64_MAX;
    char *end = nullptr;
    double v = strtod(e, &end);
    if (end && (*end == 'K' || *end == 'k')) v *= 1024.0;
    if (end && (*end == 'M' || *end == 'm')) v *= 1024.0 * 1024.0;
    if (end && (*end == 'G' || *end == 'g')) v *= 1024.0 * 1024.0 * 1024.0;
    return v < 0 ? 0ull : (uint64_t)v;
}
// reserve `need` bytes of the device's arena budget (false: past it)
bool arena_budget_take(int dev, uint64_t need) {
    const uint64_t cap = arena_keep_max();
    std::lock_guard<std::mutex> lk(g_cache_mu);
    uint64_t &k = g_kept_dev[dev];
    if (cap != UINT64_MAX && k + need > cap) return false;
    k += need;
    return true;
}
void arena_budget_give(int dev, uint64_t n) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    uint64_t &k = g_kept_dev[dev];
    k = k > n ? k - n : 0ull;
}
std::vector<const pf_ctx_t *> g_keep_on;    // contexts whose -u pre-pass keeps its arenas

bool cache_enabled(const pf_ctx_t *ctx) {
    const char *e = getenv("PF_FETCH_CACHE");
    const bool off = e && !strcmp(e, "0");
    if (off) return false;
    std::lock_guard<std::mutex> lk(g_cache_mu);
    return std::find(g_keep_on.begin(), g_keep_on.end(), ctx) != g_keep_on.end();
}

// PF_FETCH_CACHE_SCOPE=ctx: an arena serves only the context that kept it,
// and the driver treats every context as a device of its own (the -u
// pre-pass runs on all of them): the multi-GPU affinity of window jobs,
// rehearsed on one GPU (tests).
extern "C" int pf_fetch_cache_scope_ctx(void) {
    const char *e = getenv("PF_FETCH_CACHE_SCOPE");
    return e && !strcmp(e, "ctx") ? 1 : 0;
}

// An arena kept by any context of the same device serves this one: the
// driver's contexts of one GPU (PF_DEV_CONTEXTS) share its HBM, and the -u
// pre-pass that wrote the arenas has finished (its jobs joined) before the
// window jobs look them up.
// ... whose piece holds the regions [lo, hi) of a fetch (lo > hi: any piece)
const ArenaCache *cache_find(const pf_ctx_t *ctx, const char *path, const struct stat &s, int32_t tid, int64_t lo,
                             int64_t hi) {
    const int dev = pf_ctx_device((const pf_ctx *)ctx);
    const bool by_ctx = pf_fetch_cache_scope_ctx() != 0;
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (const ArenaCache *c : g_cache)
        if ((c->ctx == ctx || (!by_ctx && pf_ctx_device((const pf_ctx *)c->ctx) == dev)) && c->tid == tid &&
            (lo > hi || (c->pbeg <= lo && hi <= c->pend)) &&
            c->fsize == (uint64_t)s.st_size && c->mt_s == (int64_t)s.st_mtim.tv_sec &&
            c->mt_ns == (int64_t)s.st_mtim.tv_nsec && c->path == path)
            return c;
    return nullptr;
}

// The first of ctxs[0, n) that a kept arena of (path, contig tid) whose piece
// holds [lo, hi) would serve, or -1: the home of a window job (pf_pipeline.c).
extern "C" int pf_fetch_cache_home_range(pf_ctx_t *const *ctxs, int n, const char *path, int32_t tid, int64_t lo,
                                         int64_t hi) {
    struct stat s;
    if (!path || stat(path, &s) != 0) return -1;
    for (int i = 0; i < n; i++)
        if (cache_find(ctxs[i], path, s, tid, lo, hi)) return i;
    return -1;
}
extern "C" int pf_fetch_cache_home(pf_ctx_t *const *ctxs, int n, const char *path, int32_t tid) {
    return pf_fetch_cache_home_range(ctxs, n, path, tid, 1, 0);
}

// The plan's blocks from a kept arena: per run, the kept blocks from its
// first address while they lie whole inside the run -- the blocks the scan of
// the file bytes would find.  False when the kept arena does not cover a run
// (its blocks stop before the run does, short of EOF).
bool plan_from_cache_(const ArenaCache &C, Plan &P, uint64_t fsize);
bool plan_from_cache(const ArenaCache &C, Plan &P, uint64_t fsize) {
    if (plan_from_cache_(C, P, fsize)) return true;
    P.blk.clear(); P.caddr.clear(); P.bsize.clear();     // the file path scans from scratch
    for (Range &R : P.runs) { R.b0 = R.b1 = 0; R.end_addr = 0; R.to_eof = false; R.scan = 0; }
    P.arena = 0;
    return false;
}
bool plan_from_cache_(const ArenaCache &C, Plan &P, uint64_t fsize) {
    P.blk.clear(); P.caddr.clear(); P.bsize.clear();
    const size_t n = C.caddr.size();
    for (uint32_t ri = 0; ri < P.runs.size(); ri++) {
        Range &R = P.runs[ri];
        R.b0 = (uint32_t)P.blk.size();
        size_t i = (size_t)(std::lower_bound(C.caddr.begin(), C.caddr.end(), R.f0) - C.caddr.begin());
        if (i >= n || C.caddr[i] != R.f0) return false;
        uint64_t e = R.f0;
        for (; i < n && C.caddr[i] == e && C.caddr[i] + C.bsize[i] <= R.f1; i++) {
            pf_bgzf_blk b;
            memset(&b, 0, sizeof b);
            b.out_off = C.out_off[i];
            b.isize = C.isize[i];
            b.run = ri;
            P.blk.push_back(b);
            P.caddr.push_back(e);
            P.bsize.push_back(C.bsize[i]);
            e += C.bsize[i];
        }
        // past the run: the next block is known and does not fit, or the file
        // ends, or the kept run's scan stopped at e within a range that
        // reached at least as far as this run's
        const bool next_known = i < n && C.caddr[i] == e;
        if (!next_known && e < fsize && e + 18 <= R.f1 && !(e > R.f0 && R.f1 <= C.run_f1[C.run[i - 1]])) return false;
        R.b1 = (uint32_t)P.blk.size();
        R.end_addr = e;
        R.to_eof = e >= fsize;
    }
    P.arena = C.arena;
    return true;
}

// The compressed bytes are staged in the context's pinned buffer (grown on
// demand and reused by every fetch of that context: pinning costs about as
// much as the copy it enables).  One fetch runs on a context at a time, so
// the buffer needs no lock; two contexts never share one.

// the gathered small fields, host side
struct Small {
    std::vector<uint16_t> flag;
    std::vector<uint8_t> mapq, hp, st;
    std::vector<uint32_t> pos, l_qseq, ncig, mm_len, ml_len, qn_len, md_len, rlen, nins;
    std::vector<float> de;
    std::vector<int32_t> hp_tag;
    void resize(size_t n) {
        flag.resize(n); mapq.resize(n); hp.resize(n); st.resize(n); pos.resize(n); l_qseq.resize(n);
        ncig.resize(n); mm_len.resize(n); ml_len.resize(n); qn_len.resize(n); md_len.resize(n); rlen.resize(n);
        nins.resize(n);
        de.resize(n); hp_tag.resize(n);
    }
};

int read_range(int fd, uint64_t off, uint64_t n, uint8_t *dst) {
    uint64_t got = 0;
    while (got < n) {
        const ssize_t k = pread(fd, dst + got, (size_t)std::min<uint64_t>(n - got, 1ull << 30), (off_t)(off + got));
        if (k < 0) { if (errno == EINTR) continue; return -1; }
        if (k == 0) break;
        got += (uint64_t)k;
    }
    return got == n ? 0 : -1;
}

}  // namespace

struct pf_bam_dev_fetch_own {
    pf_bam_dev_fetch_t pub;
    std::vector<uint8_t> read_hp;
    std::vector<uint32_t> win_rec_off, win_n, win_status;
    std::vector<uint64_t> qn_off, md_off;
    std::vector<char> qn, md;
    Small s;
};

extern "C" void pf_bam_dev_fetch_free(pf_bam_dev_fetch_t *f) { delete reinterpret_cast<pf_bam_dev_fetch_own *>(f); }

// device fill of a record-level batch: gather the large arrays from the arena
struct DevFill {
    const uint8_t *arena;
    const uint32_t *sel;
    uint64_t n;
    pf_recs_dev R;
    const uint64_t *d_cig_off, *d_mm_off, *d_ml_off;
    hipStream_t st;
};
static int dev_fill(void *user, pf_ctx *ctx, pf_load_dev *ld, const uint64_t *seq_off, uint64_t seq_bytes) {
    (void)ctx; (void)seq_bytes;
    DevFill *f = static_cast<DevFill *>(user);
    if (!f->n) return PF_OK;
    // the batch's seq_off is on the device already (ld->seq_off)
    hipLaunchKernelGGL(pf_gather_big, dim3((unsigned)((f->n + 3) / 4)), dim3(256), 0, f->st, f->arena, f->sel, f->n,
                       f->R, ld->cigar_off, const_cast<uint32_t *>(ld->cigar), ld->seq_off,
                       const_cast<uint8_t *>(ld->seq), ld->mm_off, const_cast<uint8_t *>(ld->mm), ld->ml_off,
                       const_cast<uint8_t *>(ld->ml), nullptr, nullptr, nullptr, nullptr);
    (void)seq_off;
    if (hipGetLastError() != hipSuccess) return PF_ERR_HIP;
    return hipStreamSynchronize(f->st) == hipSuccess ? PF_OK : PF_ERR_HIP;
}

// what the device fetch hands its sink: the arena, the selected records
// (indices into the decoded record arrays, window by window) and their small
// fields on the host; device memory stays valid until the sink returns
struct FetchOut {
    const uint8_t *arena;
    const uint32_t *sel;
    uint64_t n;
    pf_recs_dev R;
    const Small *S;
    hipStream_t st;
    DevBuf *D;
};

// The device fetch of W regions [beg, end) of tid (reads: the -u pre-pass
// records); F receives window counts, qnames and statistics; sink builds what
// the caller needs from the gathered records.
template <typename Sink>
static int dev_fetch(pf_ctx_t *ctx, pf_bam_t *bam, int32_t tid, uint32_t W, const int64_t *beg, const int64_t *end,
                     uint32_t reads, uint32_t max_win_recs, pf_bam_dev_fetch_own *F, Sink &&sink,
                     ArenaCache *keep = nullptr) {
    const char *path = pf_bam_path(bam);
    if (!path || tid < 0) return PF_ERR_ARG;
    const double t_start = now_ms();
    // ---- chunk lists (the BAI query of every window)
    std::vector<uint64_t> uv;
    std::vector<uint32_t> wc(W + 1, 0);
    for (uint32_t w = 0; w < W; w++) {
        const int64_t n = pf_bam_query_chunks(bam, tid, beg[w], end[w], nullptr, 0);
        if (n < 0) return (int)n;
        const size_t o = uv.size();
        uv.resize(o + 2 * (size_t)n);
        if (n && pf_bam_query_chunks(bam, tid, beg[w], end[w], uv.data() + o, (uint64_t)n) != n) return PF_ERR_INTERNAL;
        wc[w + 1] = wc[w] + (uint32_t)n;
    }
    const uint32_t NC = wc[W];
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    struct stat stt;
    if (fstat(fd, &stt) != 0) { close(fd); return -1; }
    const uint64_t fsize = (uint64_t)stt.st_size;
    int64_t lo_all = INT64_MAX, hi_all = 0;               // the regions' union: the kept piece must hold it
    for (uint32_t w = 0; w < W; w++) { lo_all = std::min(lo_all, beg[w]); hi_all = std::max(hi_all, end[w]); }
    const ArenaCache *AC = W ? cache_find(ctx, path, stt, tid, lo_all, hi_all) : nullptr;
    hipStream_t st = pf_ctx_stream((const pf_ctx *)ctx);
    if (hipSetDevice(pf_ctx_device((const pf_ctx *)ctx)) != hipSuccess) { close(fd); return PF_ERR_HIP; }
    memset(&F->pub, 0, sizeof F->pub);
    int rc = PF_OK;
    bool done = false;                    // an attempt covered every window and ran the sink
    uint64_t ext = 4ull << 16;            // bytes read past a chunk's last block (records spanning blocks)
    for (int attempt = 0; attempt < 8; attempt++) {
        DevBuf D;
        D.st = st;
        Plan P;
        double t0 = now_ms();
        // ---- byte ranges: [u >> 16, (v >> 16) + ext) per chunk, merged
        std::vector<std::pair<uint64_t, uint64_t>> rq;
        rq.reserve(NC);
        for (uint32_t c = 0; c < NC; c++) {
            const uint64_t a0 = uv[2 * c] >> 16, a1 = std::min(fsize, (uv[2 * c + 1] >> 16) + ext);
            if (a0 < fsize) rq.push_back({a0, std::max(a1, a0 + 1)});
        }
        std::sort(rq.begin(), rq.end());
        for (auto &x : rq) {
            if (!P.runs.empty() && x.first <= P.runs.back().f1) P.runs.back().f1 = std::max(P.runs.back().f1, x.second);
            else P.runs.push_back(Range{x.first, x.second, 0, 0, 0, 0, false, 0});
        }
        uint64_t tot = 0;
        for (auto &R : P.runs) { R.buf0 = tot; tot += R.f1 - R.f0; }
        hipStream_t cs = pf_ctx_stream2((const pf_ctx *)ctx), s3 = pf_ctx_stream3((const pf_ctx *)ctx);
        D.st2 = cs;
        D.st3 = s3;
        hipEvent_t ev[8], ecp, eh[2];
        bool used[2] = {false, false};
        int nev = 0;
        for (auto &e : ev) if (hipEventCreateWithFlags(&e, 0) == hipSuccess) nev++;
        const bool ev_ok = nev == 8 && hipEventCreateWithFlags(&ecp, hipEventDisableTiming) == hipSuccess &&
                           hipEventCreateWithFlags(&eh[0], hipEventDisableTiming) == hipSuccess &&
                           hipEventCreateWithFlags(&eh[1], hipEventDisableTiming) == hipSuccess;
        if (!ev_ok) { rc = PF_ERR_HIP; break; }
        struct EvGuard {
            hipEvent_t *ev, *ecp, *eh;
            ~EvGuard() {
                for (int i = 0; i < 8; i++) (void)hipEventDestroy(ev[i]);
                (void)hipEventDestroy(*ecp); (void)hipEventDestroy(eh[0]); (void)hipEventDestroy(eh[1]);
            }
        } evg{ev, &ecp, eh};
        // per batch of blocks: its device descriptors and status words
        struct Batch { uint32_t b0, n; pf_bgzf_blk *d_blk; uint32_t *d_st; };
        std::vector<Batch> batches;
        uint8_t *d_arena = nullptr;
        // a whole-contig arena of this context holding every block of the plan
        // (the -u pre-pass's): no reads, no inflate
        const bool cached = AC && plan_from_cache(*AC, P, fsize);
        if (cached) {
            d_arena = AC->d_arena;
            if (hipEventRecord(ev[0], st) != hipSuccess || hipEventRecord(ev[1], st) != hipSuccess) { rc = PF_ERR_HIP; break; }
        }
        if (!cached) {
        // The pinned buffer holds the runs' bytes, then a two-half ring of
        // block descriptors on their way to the device.
        constexpr uint32_t RING = 16384;                                   // descriptors per half
        // A launch waits for MINB blocks, and launches alternate between two
        // streams so that one's tail overlaps the next (a wave decodes a block
        // at a few MB/s: the rate comes from blocks in flight, about one per
        // wave slot of the chip).
        constexpr uint32_t MINB = 4096;
        // The compressed bytes pass through a fixed pinned ring of NSLOT
        // segment slots on their way to d_comp (round 4; round 3 pinned a
        // buffer of the whole fetch, ~0.5 s for a 2 GB contig in a fresh
        // process -- more than reading it).  A slot holds its segment's
        // bytes behind the LB bytes before them (a copy of the previous
        // segment's tail), so a block the previous scan left incomplete --
        // it starts at most one BGZF block before the segment -- is scanned
        // from one slot, header and footer.
        constexpr uint64_t LB = 65536, PAD = 512;
        uint64_t SEG = 64ull << 20, PIECE = 4ull << 20;
        if (const char *e = getenv("PF_INGEST_SEG")) {     // tests: small segments (many slots, straddling blocks)
            SEG = std::max<uint64_t>(strtoull(e, nullptr, 10), 4096);
            PIECE = std::min(PIECE, SEG);
        }
        if (const char *e = getenv("PF_INGEST_PIECE"))     // tests: read pieces not dividing the segment
            PIECE = std::min(SEG, std::max<uint64_t>(strtoull(e, nullptr, 10), 512));
        constexpr uint32_t NSLOT = 3;
        const uint64_t slot_b = LB + SEG + PAD;
        const uint64_t ring_at = NSLOT * slot_b;
        P.comp_n = tot + PAD;
        uint8_t *stage = pf_ctx_stage((pf_ctx *)ctx, ring_at + 2ull * RING * sizeof(pf_bgzf_blk));
        uint8_t *d_comp = D.alloc<uint8_t>(P.comp_n);
        if (!stage || !d_comp) { rc = PF_ERR_NOMEM; break; }
        pf_bgzf_blk *ring = reinterpret_cast<pf_bgzf_blk *>(stage + ring_at);
        hipEvent_t eslot[NSLOT];
        bool slot_used[NSLOT] = {};
        int nes = 0;
        for (auto &e : eslot) if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) nes++;
        struct SlotEvGuard {
            hipEvent_t *e; int n;
            ~SlotEvGuard() { for (int i = 0; i < n; i++) (void)hipEventDestroy(e[i]); }
        } sevg{eslot, nes};
        if (nes != (int)NSLOT) { rc = PF_ERR_HIP; break; }
        uint64_t win0 = 0;                    // the current slot holds global [win0 - LB, win1)
        uint8_t *win_p = stage;               // host address of global win0 - LB
        auto hp = [&](uint64_t x) { return win_p + (x + LB - win0); };
        // The inflated arena is sized from the compressed bytes (BAM inflates
        // 1.5-3x); blocks past it wait for an exact arena after the reads.
        const uint64_t acap = 4 * tot + (1ull << 20);
        d_arena = D.alloc<uint8_t>(acap + 512);
        if (!d_arena) { rc = PF_ERR_NOMEM; break; }
        const double t_alloc = now_ms();                    // PF_INGEST_TRACE
        uint32_t nb_sent = 0;                 // blocks whose inflate is enqueued
        uint32_t cur = 0;                     // first run not completely scanned
        bool spill = false;                   // the arena estimate was short
        // Scan the runs' blocks up to buffer offset `front` (whole blocks only;
        // a run is complete once its last whole block is scanned).
        auto scan_to = [&](uint64_t front) -> int {
            for (; cur < P.runs.size(); cur++) {
                Range &R = P.runs[cur];
                if (R.buf0 > front) return PF_OK;
                if (R.scan == 0) R.b0 = (uint32_t)P.blk.size();
                const uint64_t len = R.f1 - R.f0, avail = std::min(len, front - R.buf0);
                uint64_t o = R.scan;
                bool end = false;
                for (;;) {
                    if (o + 18 > len) { end = true; break; }
                    if (o + 18 > avail) break;
                    const uint8_t *h = hp(R.buf0 + o);
                    if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return PF_ERR_ARG;
                    const uint32_t xlen = rd16(h + 10);
                    if (o + 12 + xlen > len) { end = true; break; }
                    if (o + 12 + xlen > avail) break;
                    uint32_t bsize = 0;
                    for (uint32_t x = 0; x + 4 <= xlen;) {
                        const uint8_t *sf = h + 12 + x;
                        const uint32_t slen = rd16(sf + 2);
                        if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) bsize = rd16(sf + 4) + 1;
                        x += 4 + slen;
                    }
                    if (bsize < 12 + xlen + 8 || bsize > 65536) return PF_ERR_ARG;
                    if (o + bsize > len) { end = true; break; }
                    if (o + bsize > avail) break;
                    pf_bgzf_blk b;
                    b.in_off = R.buf0 + o + 12 + xlen;
                    b.in_len = bsize - 12 - xlen - 8;
                    b.crc = rd32(h + bsize - 8);
                    b.isize = rd32(h + bsize - 4);
                    if (b.isize > 65536) return PF_ERR_ARG;
                    b.out_off = P.arena;
                    b.run = cur;
                    P.arena += b.isize;
                    P.blk.push_back(b);
                    P.caddr.push_back(R.f0 + o);
                    P.bsize.push_back(bsize);
                    o += bsize;
                }
                R.scan = o;
                if (!end) return PF_OK;
                R.b1 = (uint32_t)P.blk.size();
                R.end_addr = R.f0 + o;
                R.to_eof = R.end_addr >= fsize;
            }
            return PF_OK;
        };
        // Enqueue the inflate of the scanned blocks not yet sent (at least
        // MINB of them unless `last`), into `arena`:
        // descriptors through the pinned ring on the copy stream, the kernel
        // on the main stream behind the copies.
        auto send = [&](uint8_t *arena, bool last) -> int {
            if (!last && P.blk.size() - nb_sent < MINB) return PF_OK;
            while (nb_sent < P.blk.size()) {
                const uint32_t n = std::min<uint32_t>(RING, (uint32_t)P.blk.size() - nb_sent);
                const int h = (int)(batches.size() & 1);
                if (used[h] && hipEventSynchronize(eh[h]) != hipSuccess) return PF_ERR_HIP;
                pf_bgzf_blk *hb = ring + (size_t)h * RING;
                memcpy(hb, P.blk.data() + nb_sent, sizeof(pf_bgzf_blk) * n);
                Batch B{nb_sent, n, D.alloc<pf_bgzf_blk>(n), D.alloc<uint32_t>(n)};
                if (!B.d_blk || !B.d_st) return PF_ERR_NOMEM;
                if (hipMemcpyAsync(B.d_blk, hb, sizeof(pf_bgzf_blk) * n, hipMemcpyHostToDevice, cs) != hipSuccess ||
                    hipEventRecord(eh[h], cs) != hipSuccess || hipEventRecord(ecp, cs) != hipSuccess)
                    return PF_ERR_HIP;
                const hipStream_t ks = (batches.size() & 1) ? s3 : st;
                if (batches.empty() && hipEventRecord(ev[0], cs) != hipSuccess) return PF_ERR_HIP;
                if (hipStreamWaitEvent(ks, ecp, 0) != hipSuccess || hipMemsetAsync(B.d_st, 0, 4ull * n, ks) != hipSuccess)
                    return PF_ERR_HIP;
                used[h] = true;
                const int r = pf_inflate_launch((pf_ctx *)ctx, ks, d_comp, B.d_blk, P.blk.data() + nb_sent, n, arena,
                                                B.d_st, nullptr, nullptr);
                if (r) return r;
                batches.push_back(B);
                nb_sent += n;
            }
            return PF_OK;
        };
        // Parallel reads into the ring's slots in segments of <= 64 MiB
        // (pieces of <= 4 MiB on 16 threads); each segment's H2D copy runs on
        // the copy stream and its whole blocks are inflated on the main stream
        // while the next segments are read.
        {
            std::vector<std::pair<uint64_t, uint64_t>> pieces;     // (run, offset in run)
            for (uint32_t ri = 0; ri < P.runs.size(); ri++)
                for (uint64_t o = 0; o < P.runs[ri].f1 - P.runs[ri].f0; o += PIECE) pieces.push_back({ri, o});
            std::atomic<int> bad{0};
            size_t pi = 0;
            uint64_t copied = 0;
            double tr_read = 0, tr_copy = 0, tr_scan = 0, tr_send = 0;   // PF_INGEST_TRACE
            uint32_t nseg = 0;
            while (pi < pieces.size() && !bad.load() && !rc) {
                const double ta = now_ms();
                // whole pieces up to SEG bytes (a slot's capacity; pieces are
                // run-relative, so a segment over several runs ends where the
                // next piece would overflow the slot)
                const uint64_t seg0 = P.runs[pieces[pi].first].buf0 + pieces[pi].second;
                auto piece_end = [&](size_t k) {
                    const Range &R = P.runs[pieces[k].first];
                    return R.buf0 + pieces[k].second + std::min(PIECE, R.f1 - R.f0 - pieces[k].second);
                };
                size_t pe = pi + 1;
                while (pe < pieces.size() && piece_end(pe) <= seg0 + SEG) pe++;
                const uint64_t seg1 = pe < pieces.size() ? P.runs[pieces[pe].first].buf0 + pieces[pe].second : tot;
                // the slot: free once its last H2D copy is done; the previous
                // segment's tail goes in front of the new bytes
                const uint32_t sl = nseg++ % NSLOT;
                uint8_t *sp = stage + (uint64_t)sl * slot_b;
                if (slot_used[sl] && hipEventSynchronize(eslot[sl]) != hipSuccess) { bad.store(2); break; }
                const uint64_t lb = std::min(LB, seg0);
                if (lb) memcpy(sp + LB - lb, hp(seg0 - lb), lb);
                win0 = seg0;
                win_p = sp;
                std::atomic<size_t> next{pi};
                std::vector<std::thread> th;
                const size_t nt = std::min<size_t>(16, pe - pi);
                for (size_t t = 0; t < nt; t++)
                    th.emplace_back([&]() {
                        for (size_t k; (k = next.fetch_add(1)) < pe;) {
                            const Range &R = P.runs[pieces[k].first];
                            const uint64_t o = pieces[k].second, n = std::min(PIECE, R.f1 - R.f0 - o);
                            if (read_range(fd, R.f0 + o, n, hp(R.buf0 + o))) bad.store(1);
                        }
                    });
                for (auto &t : th) t.join();
                const double tb = now_ms();
                tr_read += tb - ta;
                if (bad.load()) break;
                if (pe == pieces.size()) memset(hp(tot), 0, PAD);
                const uint64_t cend = pe == pieces.size() ? tot + PAD : seg1;
                if (hipMemcpyAsync(d_comp + copied, hp(copied), cend - copied, hipMemcpyHostToDevice, cs) !=
                        hipSuccess || hipEventRecord(eslot[sl], cs) != hipSuccess) { bad.store(2); break; }
                slot_used[sl] = true;
                copied = cend;
                pi = pe;
                const double tc = now_ms();
                rc = scan_to(seg1);
                const double td = now_ms();
                if (!rc && !spill) {
                    if (P.arena > acap) spill = true;
                    else rc = send(d_arena, false);
                }
                const double te = now_ms();
                tr_copy += tc - tb; tr_scan += td - tc; tr_send += te - td;
            }
            if (getenv("PF_INGEST_TRACE"))
                fprintf(stderr, "[ingest] %zu pieces %.1f MB: plan + stage + alloc %.1f ms, read %.1f ms, copy enqueue "
                        "%.1f, scan %.1f, send %.1f\n", pieces.size(), tot / 1e6, t_alloc - t0, tr_read, tr_copy,
                        tr_scan, tr_send);
            if (!rc && bad.load()) rc = bad.load() == 1 ? -1 : PF_ERR_HIP;
            if (!rc && pieces.empty()) {
                memset(stage, 0, PAD);
                if (hipMemcpyAsync(d_comp, stage, PAD, hipMemcpyHostToDevice, cs) != hipSuccess) rc = PF_ERR_HIP;
            }
        }
        if (!rc) rc = scan_to(tot);
        if (!rc && spill) {
            // the exact arena: what was inflated moves over, the rest follows
            uint8_t *a2 = D.alloc<uint8_t>(P.arena + 512);
            if (!a2) rc = PF_ERR_NOMEM;
            const uint64_t done = nb_sent ? P.blk[nb_sent - 1].out_off + P.blk[nb_sent - 1].isize : 0;
            if (!rc && (hipEventRecord(ecp, s3) != hipSuccess || hipStreamWaitEvent(st, ecp, 0) != hipSuccess))
                rc = PF_ERR_HIP;
            if (!rc && done && hipMemcpyAsync(a2, d_arena, done, hipMemcpyDeviceToDevice, st) != hipSuccess) rc = PF_ERR_HIP;
            if (!rc && (hipEventRecord(ecp, st) != hipSuccess || hipStreamWaitEvent(s3, ecp, 0) != hipSuccess))
                rc = PF_ERR_HIP;
            d_arena = a2;
        }
        if (!rc) rc = send(d_arena, true);
        // the slots' copies are done before the staging buffer is reused --
        // on the error exits too (the context keeps the stage for its next fetch)
        if (hipStreamSynchronize(cs) != hipSuccess && !rc) rc = PF_ERR_HIP;
        if (!rc && batches.empty() && hipEventRecord(ev[0], st) != hipSuccess) rc = PF_ERR_HIP;
        if (!rc && (hipEventRecord(ecp, cs) != hipSuccess || hipStreamWaitEvent(st, ecp, 0) != hipSuccess ||
                    hipEventRecord(ecp, s3) != hipSuccess || hipStreamWaitEvent(st, ecp, 0) != hipSuccess ||
                    hipEventRecord(ev[1], st) != hipSuccess))
            rc = PF_ERR_HIP;
        }
        if (rc) break;
        const double t_read = now_ms() - t0;
        if (getenv("PF_INGEST_TRACE")) fprintf(stderr, "[ingest] t_read %.1f ms\n", t_read);
        const uint32_t NB = (uint32_t)P.blk.size(), NR = (uint32_t)P.runs.size();
        // ---- chunks -> arena positions; chain starts per run
        auto find_blk = [&](uint64_t addr) -> int64_t {
            const auto it = std::lower_bound(P.caddr.begin(), P.caddr.end(), addr);
            return (it != P.caddr.end() && *it == addr) ? (int64_t)(it - P.caddr.begin()) : -1;
        };
        std::vector<pf_chunk_dev> ch(NC);
        std::vector<pf_run_dev> rd(NR);
        for (uint32_t ri = 0; ri < NR; ri++) {
            const Range &R = P.runs[ri];
            rd[ri].a0 = R.b0 < R.b1 ? P.blk[R.b0].out_off : P.arena;
            rd[ri].a1 = R.b0 < R.b1 ? P.blk[R.b1 - 1].out_off + P.blk[R.b1 - 1].isize : rd[ri].a0;
            rd[ri].chain_start = UINT64_MAX;
            rd[ri].to_eof = R.to_eof ? 1u : 0u;
            rd[ri].stop_pos = 0;
            rd[ri].rec0 = rd[ri].n_rec = rd[ri].stop = 0;
        }
        bool more = false;
        for (uint32_t c = 0; c < NC && !rc; c++) {
            const uint64_t u = uv[2 * c], v = uv[2 * c + 1];
            const int64_t bu = find_blk(u >> 16);
            if (bu < 0 || (u & 0xFFFF) > P.blk[bu].isize) {
                if ((u >> 16) >= fsize) { ch[c].u = ch[c].v = 0; ch[c].run = 0; continue; }
                rc = PF_ERR_ARG;
                break;
            }
            const uint32_t ri = P.blk[bu].run;
            ch[c].u = P.blk[bu].out_off + (u & 0xFFFF);
            ch[c].run = ri;
            const int64_t bv = find_blk(v >> 16);
            if (bv >= 0 && P.blk[bv].run == ri && (v & 0xFFFF) <= P.blk[bv].isize) ch[c].v = P.blk[bv].out_off + (v & 0xFFFF);
            else if ((v >> 16) == P.runs[ri].end_addr && (v & 0xFFFF) == 0) ch[c].v = rd[ri].a1;
            else if ((v >> 16) >= P.runs[ri].end_addr && !P.runs[ri].to_eof) { more = true; ch[c].v = rd[ri].a1; }
            else ch[c].v = rd[ri].a1;                                   // past EOF: read to the end
            if (ch[c].u < ch[c].v) rd[ri].chain_start = std::min(rd[ri].chain_start, ch[c].u);
        }
        if (rc) break;
        if (more) { ext *= 4; continue; }
        for (auto &R : rd) if (R.chain_start == UINT64_MAX) R.chain_start = R.a1;
        // chain segments: each run's chain cut at the chunk starts (record
        // boundaries by the index's construction), walked in parallel
        std::vector<pf_seg_dev> sg;
        {
            std::vector<std::vector<uint64_t>> starts(NR);
            for (uint32_t c = 0; c < NC; c++)
                if (ch[c].u < ch[c].v) starts[ch[c].run].push_back(ch[c].u);
            for (uint32_t ri = 0; ri < NR; ri++) {
                auto &v = starts[ri];
                v.push_back(rd[ri].chain_start);
                std::sort(v.begin(), v.end());
                v.erase(std::unique(v.begin(), v.end()), v.end());
                for (size_t k = 0; k < v.size(); k++) {
                    pf_seg_dev g;
                    memset(&g, 0, sizeof g);
                    g.s = v[k];
                    g.last = k + 1 == v.size();
                    g.e = g.last ? rd[ri].a1 : v[k + 1];
                    g.a1 = rd[ri].a1;
                    g.run = ri;
                    g.live = 1;
                    sg.push_back(g);
                }
            }
        }
        const uint32_t NS_ = (uint32_t)sg.size();
        std::vector<pf_win_dev> wd(W);
        for (uint32_t w = 0; w < W; w++) {
            wd[w].beg = beg[w]; wd[w].end = end[w]; wd[w].c0 = wc[w]; wd[w].c1 = wc[w + 1];
            wd[w].tid = tid; wd[w].skip = 0; wd[w].reads = (uint16_t)reads; wd[w].out = 0;
        }
        // ---- tables of the later stages (the inflate is enqueued already)
        t0 = now_ms();
        pf_run_dev *d_run = D.alloc<pf_run_dev>(NR);
        pf_seg_dev *d_sg = D.alloc<pf_seg_dev>(NS_);
        pf_chunk_dev *d_ch = D.alloc<pf_chunk_dev>(NC);
        pf_win_dev *d_win = D.alloc<pf_win_dev>(W);
        uint32_t *d_wn = D.alloc<uint32_t>(2ull * W);
        if (!d_run || !d_sg || !d_ch || !d_win || !d_wn) { rc = PF_ERR_NOMEM; break; }
        auto evdone = [&]() {};
        bool ok = hipMemsetAsync(d_arena + P.arena, 0, 512, st) == hipSuccess &&
                  hipMemcpyAsync(d_sg, sg.data(), sizeof(pf_seg_dev) * NS_, hipMemcpyHostToDevice, st) == hipSuccess &&
                  hipMemcpyAsync(d_ch, ch.data(), sizeof(pf_chunk_dev) * NC, hipMemcpyHostToDevice, st) == hipSuccess &&
                  hipMemcpyAsync(d_win, wd.data(), sizeof(pf_win_dev) * W, hipMemcpyHostToDevice, st) == hipSuccess &&
                  hipEventRecord(ev[2], st) == hipSuccess;
        // ---- chain: count, offsets, write
        if (ok && NS_) {
            hipLaunchKernelGGL(pf_chain, dim3((NS_ + 63) / 64), dim3(64), 0, st, d_arena, d_sg, NS_, (uint64_t *)nullptr);
            ok = hipGetLastError() == hipSuccess;
        }
        std::vector<uint32_t> bst(NB);
        for (const Batch &B : batches)
            ok = ok && hipMemcpyAsync(bst.data() + B.b0, B.d_st, 4ull * B.n, hipMemcpyDeviceToHost, st) == hipSuccess;
        ok = ok && hipMemcpyAsync(sg.data(), d_sg, sizeof(pf_seg_dev) * NS_, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
        if (!ok) { evdone(); rc = PF_ERR_HIP; break; }
        for (uint32_t i = 0; i < NB; i++)
            if (bst[i]) {
                fprintf(stderr, "[E::pomfret_amd] BGZF block at file offset %llu: device inflate status %u\n",
                        (unsigned long long)P.caddr[i], bst[i]);
                rc = PF_ERR_ARG;
                break;
            }
        if (rc) { evdone(); break; }
        // per run: its segments in order; a segment that stopped early ends the
        // run's chain there (the later segments' records are not reachable by
        // a serial walk either)
        uint64_t NRec = 0;
        for (uint32_t k = 0; k < NS_;) {
            const uint32_t ri = sg[k].run;
            pf_run_dev &R = rd[ri];
            R.rec0 = (uint32_t)NRec;
            R.n_rec = 0;
            bool dead = false;
            for (; k < NS_ && sg[k].run == ri; k++) {
                pf_seg_dev &g = sg[k];
                g.live = dead ? 0u : 1u;
                if (dead) continue;
                g.rec0 = (uint32_t)(NRec + R.n_rec);
                R.n_rec += g.n;
                if (g.last || g.stop != PF_CHAIN_END) {
                    R.stop = g.stop;
                    R.stop_pos = g.stop_pos;
                    dead = !g.last;
                }
            }
            NRec += R.n_rec;
        }
        for (uint32_t ri = 0; ri < NR; ri++)              // runs without segments (no chunk of theirs reads records)
            if (rd[ri].chain_start >= rd[ri].a1) { rd[ri].n_rec = 0; rd[ri].stop = PF_CHAIN_END; rd[ri].stop_pos = rd[ri].a1; }
        if (NRec >= (1ull << 32)) { evdone(); rc = PF_ERR_LIMIT; break; }
        // the record arrays, one allocation
        pf_recs_dev Rv;
        {
            const uint64_t n = NRec ? NRec : 1, a8 = (8 * n + 255) & ~255ull, a4 = (4 * n + 255) & ~255ull,
                           a2 = (2 * n + 255) & ~255ull, a1 = (n + 255) & ~255ull;
            uint8_t *m = D.alloc<uint8_t>(8 * a8 + 13 * a4 + a2 + 3 * a1);
            if (!m) { evdone(); rc = PF_ERR_NOMEM; break; }
            auto take = [&](uint64_t bytes) { uint8_t *r = m; m += bytes; return r; };
            Rv.pos = (uint64_t *)take(a8); Rv.cig = (uint64_t *)take(a8); Rv.seq = (uint64_t *)take(a8);
            Rv.qn = (uint64_t *)take(a8); Rv.mm = (uint64_t *)take(a8); Rv.ml = (uint64_t *)take(a8);
            Rv.md = (uint64_t *)take(a8); take(a8);
            Rv.bs = (uint32_t *)take(a4); Rv.l_qseq = (uint32_t *)take(a4); Rv.ncig = (uint32_t *)take(a4);
            Rv.rlen = (uint32_t *)take(a4); Rv.qn_len = (uint32_t *)take(a4); Rv.mm_len = (uint32_t *)take(a4);
            Rv.ml_len = (uint32_t *)take(a4); Rv.md_len = (uint32_t *)take(a4); Rv.nins = (uint32_t *)take(a4);
            Rv.tid = (int32_t *)take(a4); Rv.rpos = (int32_t *)take(a4); Rv.hp_tag = (int32_t *)take(a4);
            Rv.de = (float *)take(a4);
            Rv.flag = (uint16_t *)take(a2);
            Rv.mapq = take(a1); Rv.hp = take(a1); Rv.st = take(a1);
        }
        ok = hipMemcpyAsync(d_run, rd.data(), sizeof(pf_run_dev) * NR, hipMemcpyHostToDevice, st) == hipSuccess &&
             hipMemcpyAsync(d_sg, sg.data(), sizeof(pf_seg_dev) * NS_, hipMemcpyHostToDevice, st) == hipSuccess &&
             hipEventRecord(ev[3], st) == hipSuccess;
        if (ok && NS_) {
            hipLaunchKernelGGL(pf_chain, dim3((NS_ + 63) / 64), dim3(64), 0, st, d_arena, d_sg, NS_, Rv.pos);
            ok = hipGetLastError() == hipSuccess;
        }
        if (ok && NRec) {
            hipLaunchKernelGGL(pf_recdec, dim3((unsigned)((NRec + 3) / 4)), dim3(256), 0, st, d_arena, (uint32_t)NRec, Rv);
            ok = hipGetLastError() == hipSuccess;
        }
        ok = ok && hipEventRecord(ev[4], st) == hipSuccess;
        if (ok && W) {
            hipLaunchKernelGGL(pf_select, dim3((W + 3) / 4), dim3(256), 0, st, d_win, W, d_ch, d_run, Rv, 0u, d_wn,
                               d_wn + W, (uint32_t *)nullptr);
            ok = hipGetLastError() == hipSuccess;
        }
        std::vector<uint32_t> wn(2ull * W);
        ok = ok && hipMemcpyAsync(wn.data(), d_wn, 8ull * W, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
        if (!ok) { evdone(); rc = PF_ERR_HIP; break; }
        bool need_more = false;
        uint64_t n_trunc = 0;
        for (uint32_t w = 0; w < W; w++) {
            if (wn[W + w] == PF_WIN_MORE) need_more = true;
            else if (wn[W + w] == PF_WIN_ERR) rc = PF_ERR_ARG;
            else if (wn[W + w] == PF_WIN_TRUNC) n_trunc++;
        }
        if (rc) { evdone(); break; }
        if (need_more) { evdone(); ext *= 4; continue; }
        // ---- record lists: windows over the limit are emptied
        F->win_n.assign(wn.begin(), wn.begin() + W);
        F->win_status.assign(wn.begin() + W, wn.end());
        F->win_rec_off.assign(W + 1, 0);
        for (uint32_t w = 0; w < W; w++) {
            const bool skip = max_win_recs && wn[w] > max_win_recs;
            wd[w].skip = skip ? 1u : 0u;
            wd[w].out = F->win_rec_off[w];
            F->win_rec_off[w + 1] = F->win_rec_off[w] + (skip ? 0u : wn[w]);
        }
        const uint64_t NS = F->win_rec_off[W];
        if (NS >= (1ull << 32)) { evdone(); rc = PF_ERR_LIMIT; break; }
        uint32_t *d_sel = D.alloc<uint32_t>(NS);
        if (!d_sel) { evdone(); rc = PF_ERR_NOMEM; break; }
        ok = hipMemcpyAsync(d_win, wd.data(), sizeof(pf_win_dev) * W, hipMemcpyHostToDevice, st) == hipSuccess;
        if (ok && W) {
            hipLaunchKernelGGL(pf_select, dim3((W + 3) / 4), dim3(256), 0, st, d_win, W, d_ch, d_run, Rv, 1u, d_wn,
                               d_wn + W, d_sel);
            ok = hipGetLastError() == hipSuccess;
        }
        // ---- small fields of the selected records -> host
        Small &S = F->s;
        S.resize(NS);
        uint16_t *g_flag = D.alloc<uint16_t>(NS);
        uint8_t *g_mapq = D.alloc<uint8_t>(NS), *g_hp = D.alloc<uint8_t>(NS), *g_st = D.alloc<uint8_t>(NS);
        uint32_t *g32 = D.alloc<uint32_t>(9 * NS);
        float *g_de = D.alloc<float>(NS);
        int32_t *g_hpt = D.alloc<int32_t>(NS);
        if (!g_flag || !g_mapq || !g_hp || !g_st || !g32 || !g_de || !g_hpt) { evdone(); rc = PF_ERR_NOMEM; break; }
        if (ok && NS) {
            hipLaunchKernelGGL(pf_gather_small, dim3((unsigned)((NS + 255) / 256)), dim3(256), 0, st, d_sel, NS, Rv,
                               g_flag, g_mapq, g32, g32 + NS, g_de, g_hp, g_hpt, g32 + 2 * NS, g32 + 3 * NS,
                               g32 + 4 * NS, g32 + 5 * NS, g32 + 6 * NS, g32 + 7 * NS, g_st, g32 + 8 * NS);
            ok = hipGetLastError() == hipSuccess;
        }
        ok = ok && hipEventRecord(ev[5], st) == hipSuccess;
        std::vector<uint32_t> h32(9 * NS);
        ok = ok && hipMemcpyAsync(S.flag.data(), g_flag, 2 * NS, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipMemcpyAsync(S.mapq.data(), g_mapq, NS, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipMemcpyAsync(S.hp.data(), g_hp, NS, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipMemcpyAsync(S.st.data(), g_st, NS, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipMemcpyAsync(h32.data(), g32, 36 * NS, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipMemcpyAsync(S.de.data(), g_de, 4 * NS, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipMemcpyAsync(S.hp_tag.data(), g_hpt, 4 * NS, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
        if (!ok) { evdone(); rc = PF_ERR_HIP; break; }
        memcpy(S.pos.data(), h32.data(), 4 * NS);
        memcpy(S.l_qseq.data(), h32.data() + NS, 4 * NS);
        memcpy(S.ncig.data(), h32.data() + 2 * NS, 4 * NS);
        memcpy(S.mm_len.data(), h32.data() + 3 * NS, 4 * NS);
        memcpy(S.ml_len.data(), h32.data() + 4 * NS, 4 * NS);
        memcpy(S.qn_len.data(), h32.data() + 5 * NS, 4 * NS);
        memcpy(S.md_len.data(), h32.data() + 6 * NS, 4 * NS);
        memcpy(S.rlen.data(), h32.data() + 7 * NS, 4 * NS);
        memcpy(S.nins.data(), h32.data() + 8 * NS, 4 * NS);
        // ---- qnames (and MD) -> host
        F->qn_off.assign(NS + 1, 0);
        F->md_off.assign(NS + 1, 0);
        for (uint64_t i = 0; i < NS; i++) {
            F->qn_off[i + 1] = F->qn_off[i] + S.qn_len[i];
            F->md_off[i + 1] = F->md_off[i] + S.md_len[i];
        }
        F->qn.resize(F->qn_off[NS] + 1);
        uint64_t *d_qo = D.alloc<uint64_t>(NS + 1);
        uint8_t *d_qn = D.alloc<uint8_t>(F->qn_off[NS] + 1);
        if (!d_qo || !d_qn) { evdone(); rc = PF_ERR_NOMEM; break; }
        ok = hipMemcpyAsync(d_qo, F->qn_off.data(), 8 * (NS + 1), hipMemcpyHostToDevice, st) == hipSuccess;
        if (ok && NS) {
            hipLaunchKernelGGL(pf_gather_big, dim3((unsigned)((NS + 3) / 4)), dim3(256), 0, st, d_arena, d_sel, NS, Rv,
                               (const uint64_t *)nullptr, (uint32_t *)nullptr, (const uint64_t *)nullptr,
                               (uint8_t *)nullptr, (const uint64_t *)nullptr, (uint8_t *)nullptr,
                               (const uint64_t *)nullptr, (uint8_t *)nullptr, d_qo, d_qn, (const uint64_t *)nullptr,
                               (uint8_t *)nullptr);
            ok = hipGetLastError() == hipSuccess;
        }
        ok = ok && hipMemcpyAsync(F->qn.data(), d_qn, F->qn_off[NS], hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
        if (!ok) { evdone(); rc = PF_ERR_HIP; break; }
        // ---- the caller's product of the gathered records
        ok = hipEventRecord(ev[6], st) == hipSuccess;
        {
            FetchOut fo{d_arena, d_sel, NS, Rv, &S, st, &D};
            rc = ok ? sink(fo) : PF_ERR_HIP;
        }
        ok = hipEventRecord(ev[7], st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
        float ms_inf = 0, ms_chain = 0, ms_dec = 0, ms_sel = 0, ms_build = 0;
        if (ok) {
            (void)hipEventElapsedTime(&ms_inf, ev[0], ev[1]);
            (void)hipEventElapsedTime(&ms_chain, ev[2], ev[3]);
            (void)hipEventElapsedTime(&ms_dec, ev[3], ev[4]);
            (void)hipEventElapsedTime(&ms_sel, ev[4], ev[5]);
            (void)hipEventElapsedTime(&ms_build, ev[6], ev[7]);
            (void)hipGetLastError();
        }
        evdone();
        if (rc) break;
        pf_bam_dev_fetch_t &pub = F->pub;
        pub.n_windows = W;
        pub.n_recs = NS;
        pub.win_rec_off = F->win_rec_off.data();
        pub.win_n_fetched = F->win_n.data();
        pub.qname_off = F->qn_off.data();
        pub.qname = F->qn.data();
        pub.hp_tag = F->s.hp_tag.data();
        pub.n_truncated = n_trunc;
        pub.comp_bytes = cached ? 0 : tot;           // (a kept arena: nothing read or inflated)
        pub.inflated_bytes = cached ? 0 : P.arena;
        pub.n_blocks = NB;
        pub.n_chain_recs = NRec;
        pub.ms_read = t_read;
        pub.ms_inflate = ms_inf;
        pub.ms_chain = ms_chain;
        pub.ms_decode = ms_dec;
        pub.ms_select = ms_sel;
        pub.ms_build = ms_build;
        pub.ms_total = now_ms() - t_start;
        pub.attempts = (uint32_t)attempt + 1;
        pub.from_arena = cached ? 1u : 0u;
        done = true;
        if (keep && !cached) {
            // an exact copy of the arena (the fetch's own is sized from the
            // compressed bytes), if the device keeps its reserve
            size_t fr = 0, tt = 0;
            const uint64_t need = P.arena + 512;
            uint8_t *k = nullptr;
            const int kdev = pf_ctx_device((const pf_ctx *)ctx);
            bool took = false;
            if (hipMemGetInfo(&fr, &tt) == hipSuccess && fr > need && fr - need > std::max<size_t>(tt / 3, 32ull << 30) &&
                (took = arena_budget_take(kdev, need)) && hipMalloc(&k, need) == hipSuccess) {
                if (hipMemcpyAsync(k, d_arena, need, hipMemcpyDeviceToDevice, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess) {
                    keep->ctx = ctx; keep->path = path; keep->fsize = fsize; keep->tid = tid;
                    keep->mt_s = (int64_t)stt.st_mtim.tv_sec; keep->mt_ns = (int64_t)stt.st_mtim.tv_nsec;
                    keep->d_arena = k; keep->arena = P.arena;
                    keep->caddr = P.caddr; keep->bsize = P.bsize;
                    keep->out_off.resize(NB); keep->isize.resize(NB); keep->run.resize(NB);
                    for (uint32_t i = 0; i < NB; i++) {
                        keep->out_off[i] = P.blk[i].out_off; keep->isize[i] = P.blk[i].isize; keep->run[i] = P.blk[i].run;
                    }
                    keep->run_f1.resize(NR);
                    for (uint32_t r = 0; r < NR; r++) keep->run_f1[r] = P.runs[r].f1;
                } else {
                    (void)hipFree(k);
                    k = nullptr;
                }
            }
            if (took && !k) arena_budget_give(kdev, need);
            (void)hipGetLastError();
        }
        break;
    }
    close(fd);
    pf_ctx_stage_trim((pf_ctx *)ctx, 8ull << 30);   // an outsized fetch does not stay pinned
    if (!rc && !done) {
        fprintf(stderr, "[E::pomfret_amd] device fetch: records still run past the planned blocks after 8 plans\n");
        rc = PF_ERR_LIMIT;
    }
    return rc;
}

extern "C" int pf_batch_upload_bam(pf_ctx_t *ctx, const pf_cfg_t *cfg, const pf_load_cfg_t *lc, pf_bam_t *bam,
                                   const char *chrom, uint32_t W, const uint32_t *ws, const uint32_t *we,
                                   uint32_t readback, uint32_t max_win_recs, pf_dbatch_t **out,
                                   pf_bam_dev_fetch_t **fetch_out) {
    if (!ctx || !cfg || !lc || !bam || !chrom || !out || !fetch_out || (W && (!ws || !we))) return PF_ERR_ARG;
    *out = nullptr;
    *fetch_out = nullptr;
    // the region string load_reads_given_interval builds (1053-1054):
    // chrom:max(s-rb,0)-(e+rb), htslib's 0-based [max(b-1, 0), E)
    std::vector<int64_t> beg(W), end(W);
    for (uint32_t w = 0; w < W; w++) {
        const int64_t s = (int32_t)ws[w], e = (int32_t)we[w], rb = (int32_t)readback;
        const int64_t b1 = s - rb > 0 ? s - rb : 0;
        beg[w] = b1 > 0 ? b1 - 1 : 0;
        end[w] = e + rb;
    }
    pf_bam_dev_fetch_own *F = new pf_bam_dev_fetch_own();
    int rc = dev_fetch(ctx, bam, pf_bam_tid(bam, chrom), W, beg.data(), end.data(), 0u, max_win_recs, F,
                       [&](FetchOut &fo) -> int {
        // the record-level batch: sizes on the host, large arrays gathered on the device
        const Small &S = *fo.S;
        const uint64_t NS = fo.n;
        std::vector<uint64_t> cig_off(NS + 1, 0), mm_off(NS + 1, 0), ml_off(NS + 1, 0);
        for (uint64_t i = 0; i < NS; i++) {
            cig_off[i + 1] = cig_off[i] + S.ncig[i];
            mm_off[i + 1] = mm_off[i] + S.mm_len[i];
            ml_off[i + 1] = ml_off[i] + S.ml_len[i];
        }
        pf_aln_batch_t a;
        memset(&a, 0, sizeof a);
        a.n_windows = W;
        a.n_recs = (uint32_t)NS;
        a.win_start = ws; a.win_end = we; a.win_rec_off = F->win_rec_off.data();
        a.flag = S.flag.data(); a.mapq = S.mapq.data(); a.pos = S.pos.data(); a.l_qseq = S.l_qseq.data();
        a.de = S.de.data(); a.hp = S.hp.data();
        a.cigar_off = cig_off.data(); a.mm_off = mm_off.data(); a.ml_off = ml_off.data();
        DevFill df{fo.arena, fo.sel, NS, fo.R, nullptr, nullptr, nullptr, fo.st};
        pf_aln_fill_t fl{dev_fill, &df};
        return pf_aln_build(ctx, cfg, lc, &a, &fl, out);
    });
    if (rc || !*out) {
        if (*out) { pf_batch_free(*out); *out = nullptr; }
        delete F;
        return rc ? rc : PF_ERR_INTERNAL;
    }
    *fetch_out = &F->pub;
    return PF_OK;
}

// Position pieces of one contig for whole-contig device fetches, each of
// about piece_bytes of compressed BAM (the contig's index chunks span
// [c0, c1) of the file): K pieces of equal reference length; a record belongs
// to the piece its start falls in.  piece_bytes 0: PF_FETCH_PIECE_BYTES or
// 4 GiB (tests force several pieces on small files with the variable).
extern "C" uint64_t pf_bam_contig_pieces(pf_bam_t *bam, int32_t tid, uint64_t piece_bytes, int64_t *step) {
    if (!piece_bytes)
        if (const char *e = getenv("PF_FETCH_PIECE_BYTES")) piece_bytes = strtoull(e, nullptr, 10);
    if (!piece_bytes) piece_bytes = 4ull << 30;
    const int64_t nc = pf_bam_query_chunks(bam, tid, 0, INT64_MAX, nullptr, 0);
    std::vector<uint64_t> uv(2 * (size_t)std::max<int64_t>(nc, 0));
    uint64_t c0 = UINT64_MAX, c1 = 0;
    if (nc > 0 && pf_bam_query_chunks(bam, tid, 0, INT64_MAX, uv.data(), (uint64_t)nc) == nc)
        for (int64_t c = 0; c < nc; c++) { c0 = std::min(c0, uv[2 * c] >> 16); c1 = std::max(c1, uv[2 * c + 1] >> 16); }
    const uint32_t len = pf_bam_target_len(bam, tid);
    const uint64_t K = c1 > c0 ? std::max<uint64_t>(1, std::min<uint64_t>(len ? len : 1, (c1 - c0 + piece_bytes - 1) /
                                                                                           piece_bytes)) : 1;
    *step = (int64_t)((len + K - 1) / K);
    return K;
}

// the coverage estimate's per-record rule (estimate_read_coverage_dirtyfast,
// 951-1040): a record passing flag 4/256/2048, mapq >= 5, l_qseq >= 15000
// and de <= 0.1 adds 1 to the 5 kb bins of start, start + 5000, ... < bam_endpos
static void cov_add(std::vector<uint64_t> &bins, const Small &S, uint64_t i) {
    constexpr uint32_t MOD = 5000;
    if ((S.flag[i] & (4u | 256u | 2048u)) || S.mapq[i] < 5 || S.l_qseq[i] < 15000) return;
    if ((double)S.de[i] > 0.1) return;
    const int32_t pos = (int32_t)S.pos[i];
    const uint32_t st = (uint32_t)pos, en = (uint32_t)(pos + (int32_t)S.rlen[i]);   // bam_endpos
    for (int64_t x = (int32_t)st; x < (int64_t)en; x += MOD) {
        const uint64_t b = (uint64_t)x / MOD;
        if (x >= 0 && b < bins.size()) bins[b]++;
    }
}

// The -u pre-pass of one contig (pf_haptag_bam) and, with cov != nullptr,
// the contig's coverage estimate from the same whole-contig fetch: every
// record of the contig is selected (the estimate's pass), the primary mapped
// ones go to K4 (the -u pass's records, which must carry MD).  *trunc is set
// when a truncated record ended the fetch (the estimate's serial pass stops
// there).
static int haptag_bam_impl(pf_ctx_t *ctx, const pf_known_vars_t *K, pf_bam_t *bam, const char *chrom,
                           pf_bam_dev_fetch_t **fetch_out, int32_t *cov, int32_t *trunc, uint32_t nb = 0,
                           const int64_t *bounds = nullptr, const int64_t *fetch_ends = nullptr) {
    if (!ctx || !K || !bam || !chrom || !fetch_out) return PF_ERR_ARG;
    *fetch_out = nullptr;
    // sam_itr_querys(idx, hdr, chrom): the whole reference, [0, HTS_POS_MAX),
    // fetched in position pieces of bounded size whose reads are concatenated
    // in BAM order (a read is taken in the piece its start falls in: the
    // coordinate-sorted records of an earlier start form a prefix of a
    // piece's overlap list); the K4 cursor chain runs on across pieces
    const int32_t tid = pf_bam_tid(bam, chrom);
    if (tid < 0) return PF_ERR_ARG;
    int64_t step = 0;
    // the pieces' bounds: the caller's (the driver places them between its
    // windows' fetch regions), else K pieces of equal reference length
    const uint64_t NP = nb ? (uint64_t)nb + 1 : pf_bam_contig_pieces(bam, tid, 0, &step);
    auto piece_beg = [&](uint64_t k) -> int64_t { return k == 0 ? 0 : nb ? bounds[k - 1] : (int64_t)k * step; };
    auto piece_end = [&](uint64_t k) -> int64_t { return k + 1 == NP ? INT64_MAX : nb ? bounds[k] : (int64_t)(k + 1) * step; };
    // a piece's fetch may reach past its bound (fetch_ends[k] >= bounds[k]:
    // the driver's windows that start in the piece and end past the bound),
    // so that its arena serves them; its reads stay those starting before the bound
    auto fetch_end = [&](uint64_t k) -> int64_t { return k + 1 < NP && fetch_ends ? fetch_ends[k] : piece_end(k); };
    const bool with_cov = cov != nullptr;
    std::vector<uint64_t> bins;
    if (with_cov) bins.assign(pf_bam_target_len(bam, tid) / 5000, 0);
    pf_bam_dev_fetch_own *F = new pf_bam_dev_fetch_own();
    F->qn_off.assign(1, 0);
    uint32_t prev_left = 0;
    double ms[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t comp = 0, infl = 0, nblk = 0, nchain = 0;
    uint32_t attempts = 0;
    int rc = PF_OK;
    for (uint64_t k = 0; k < NP && !rc; k++) {
        const int64_t beg = piece_beg(k), end = piece_end(k), fend = fetch_end(k);
        pf_bam_dev_fetch_own P;
        std::vector<uint32_t> take;                           // this piece's -u reads: selection positions
        ArenaCache *keep = cache_enabled(ctx) ? new ArenaCache() : nullptr;
        if (keep) { keep->pbeg = beg; keep->pend = fend; }
        rc = dev_fetch(ctx, bam, tid, 1, &beg, &fend, with_cov ? 0u : 1u, 0u, &P, [&](FetchOut &fo) -> int {
            const Small &S = *fo.S;
            uint64_t m = 0;                                   // records counted in an earlier piece
            if (k) while (m < fo.n && (int32_t)S.pos[m] < beg) m++;
            uint64_t me = fo.n;                               // records of a later piece (an extended fetch)
            if (fend > end) while (me > m && (int64_t)(int32_t)S.pos[me - 1] >= end) me--;
            for (uint64_t i = m; i < me; i++) {
                if (with_cov) {
                    cov_add(bins, S, i);
                    if (S.flag[i] & (4u | 256u | 2048u)) continue;              // primary mapped only (1869-1871)
                    if (!(S.st[i] & PF_REC_MD)) return PF_ERR_ARG;              // the reference asserts MD
                }
                take.push_back((uint32_t)i);
            }
            const uint64_t N = take.size();
            if (F->read_hp.size() + N >= (1ull << 32)) return PF_ERR_LIMIT;
            const size_t h0 = F->read_hp.size();
            F->read_hp.resize(h0 + N, 0);
            if (!N) return PF_OK;
            std::vector<uint32_t> start(N), endp(N), nins(N), ncig(N), mdl(N), lq(N);
            std::vector<uint64_t> co(N + 1, 0), so(N + 1, 0), mo(N + 1, 0);
            for (uint64_t i = 0; i < N; i++) {
                const uint64_t r = take[i];
                start[i] = S.pos[r];
                endp[i] = (uint32_t)((int64_t)(int32_t)S.pos[r] + (int64_t)S.rlen[r]);   // bam_endpos
                nins[i] = S.nins[r]; ncig[i] = S.ncig[r]; mdl[i] = S.md_len[r]; lq[i] = S.l_qseq[r];
                co[i + 1] = co[i] + S.ncig[r];
                so[i + 1] = so[i] + (S.l_qseq[r] + 1ull) / 2;
                mo[i + 1] = mo[i] + S.md_len[r];
            }
            DevBuf &D = *fo.D;
            hipStream_t st = fo.st;
            const uint32_t *d_take = fo.sel + m;               // contiguous unless the estimate's records are mixed in
            if (with_cov) {
                std::vector<uint32_t> sel(fo.n), ts(N);
                uint32_t *d_ts = D.alloc<uint32_t>(N);
                if (!d_ts) return PF_ERR_NOMEM;
                if (hipMemcpyAsync(sel.data(), fo.sel, 4 * fo.n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess) return PF_ERR_HIP;
                for (uint64_t i = 0; i < N; i++) ts[i] = sel[take[i]];
                if (hipMemcpyAsync(d_ts, ts.data(), 4 * N, hipMemcpyHostToDevice, st) != hipSuccess) return PF_ERR_HIP;
                d_take = d_ts;
            }
            uint32_t *d_start = D.alloc<uint32_t>(N), *d_end = D.alloc<uint32_t>(N), *d_len = D.alloc<uint32_t>(N);
            uint64_t *d_co = D.alloc<uint64_t>(N + 1), *d_so = D.alloc<uint64_t>(N + 1), *d_mo = D.alloc<uint64_t>(N + 1);
            uint32_t *d_cig = D.alloc<uint32_t>(co[N]);
            uint8_t *d_seq = D.alloc<uint8_t>(so[N] + 16), *d_md = D.alloc<uint8_t>(mo[N] + 16);
            if (!d_start || !d_end || !d_len || !d_co || !d_so || !d_mo || !d_cig || !d_seq || !d_md) return PF_ERR_NOMEM;
            bool ok = hipMemcpyAsync(d_start, start.data(), 4 * N, hipMemcpyHostToDevice, st) == hipSuccess &&
                      hipMemcpyAsync(d_end, endp.data(), 4 * N, hipMemcpyHostToDevice, st) == hipSuccess &&
                      hipMemcpyAsync(d_len, lq.data(), 4 * N, hipMemcpyHostToDevice, st) == hipSuccess &&
                      hipMemcpyAsync(d_co, co.data(), 8 * (N + 1), hipMemcpyHostToDevice, st) == hipSuccess &&
                      hipMemcpyAsync(d_so, so.data(), 8 * (N + 1), hipMemcpyHostToDevice, st) == hipSuccess &&
                      hipMemcpyAsync(d_mo, mo.data(), 8 * (N + 1), hipMemcpyHostToDevice, st) == hipSuccess;
            if (ok) {
                hipLaunchKernelGGL(pf_gather_big, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, fo.arena, d_take,
                                   N, fo.R, (const uint64_t *)d_co, d_cig, (const uint64_t *)d_so, d_seq,
                                   (const uint64_t *)nullptr, (uint8_t *)nullptr, (const uint64_t *)nullptr,
                                   (uint8_t *)nullptr, (const uint64_t *)nullptr, (uint8_t *)nullptr,
                                   (const uint64_t *)d_mo, d_md);
                ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
            }
            if (!ok) return PF_ERR_HIP;
            pf_k4_reads_host h{start.data(), endp.data(), nins.data(), ncig.data(), mdl.data()};
            pf_k4_reads_dev dv{d_start, d_end, d_co, d_cig, d_so, d_len, d_seq, d_mo, d_md};
            return pf_haptag_core(ctx, K, (uint32_t)N, h, nullptr, &dv, F->read_hp.data() + h0, &prev_left);
        }, keep);
        if (keep && keep->d_arena && !rc) {
            std::lock_guard<std::mutex> lk(g_cache_mu);
            g_cache.push_back(keep);
        } else if (keep) {
            if (keep->d_arena) (void)hipFree(keep->d_arena);
            delete keep;
        }
        if (rc) break;
        // this piece's reads' qnames
        for (const uint32_t i : take) {
            F->qn.insert(F->qn.end(), P.qn.begin() + P.qn_off[i], P.qn.begin() + P.qn_off[i + 1]);
            F->qn_off.push_back(F->qn.size());
        }
        comp += P.pub.comp_bytes; infl += P.pub.inflated_bytes; nblk += P.pub.n_blocks; nchain += P.pub.n_chain_recs;
        ms[0] += P.pub.ms_read; ms[1] += P.pub.ms_inflate; ms[2] += P.pub.ms_chain; ms[3] += P.pub.ms_decode;
        ms[4] += P.pub.ms_select; ms[5] += P.pub.ms_build; ms[6] += P.pub.ms_total;
        attempts += P.pub.attempts;
        if (P.win_status[0] == PF_WIN_TRUNC) { F->pub.n_truncated = 1; break; }   // sam_itr_next < 0 ends the loop
    }
    if (rc) { delete F; return rc; }
    if (with_cov) {
        uint64_t tot = 0;
        for (uint64_t b : bins) tot += b;
        *cov = bins.empty() ? 0 : (int32_t)(tot / bins.size());
        if (trunc) *trunc = F->pub.n_truncated ? 1 : 0;
    }
    const uint64_t N = F->read_hp.size();
    F->qn.push_back(0);
    F->win_rec_off = {0, (uint32_t)N};
    F->win_n = {(uint32_t)N};
    pf_bam_dev_fetch_t &pub = F->pub;
    pub.n_windows = 1;
    pub.n_recs = N;
    pub.win_rec_off = F->win_rec_off.data();
    pub.win_n_fetched = F->win_n.data();
    pub.qname_off = F->qn_off.data();
    pub.qname = F->qn.data();
    pub.hp_tag = nullptr;
    pub.comp_bytes = comp; pub.inflated_bytes = infl; pub.n_blocks = nblk; pub.n_chain_recs = nchain;
    pub.ms_read = ms[0]; pub.ms_inflate = ms[1]; pub.ms_chain = ms[2]; pub.ms_decode = ms[3];
    pub.ms_select = ms[4]; pub.ms_build = ms[5]; pub.ms_total = ms[6];
    pub.attempts = attempts;
    pub.read_hp = F->read_hp.data();
    *fetch_out = &F->pub;
    return PF_OK;
}

extern "C" int pf_haptag_bam(pf_ctx_t *ctx, const pf_known_vars_t *K, pf_bam_t *bam, const char *chrom,
                             pf_bam_dev_fetch_t **fetch_out) {
    return haptag_bam_impl(ctx, K, bam, chrom, fetch_out, nullptr, nullptr);
}

extern "C" int pf_haptag_bam_cov(pf_ctx_t *ctx, const pf_known_vars_t *K, pf_bam_t *bam, const char *chrom,
                                 pf_bam_dev_fetch_t **fetch_out, int32_t *cov, int32_t *truncated) {
    if (!cov || !truncated) return PF_ERR_ARG;
    return haptag_bam_impl(ctx, K, bam, chrom, fetch_out, cov, truncated);
}

extern "C" int pf_haptag_bam_pieces(pf_ctx_t *ctx, const pf_known_vars_t *K, pf_bam_t *bam, const char *chrom,
                                    uint32_t n_bounds, const int64_t *bounds, const int64_t *fetch_ends,
                                    pf_bam_dev_fetch_t **fetch_out, int32_t *cov, int32_t *truncated) {
    if (n_bounds && !bounds) return PF_ERR_ARG;
    for (uint32_t i = 0; i < n_bounds; i++) {
        if (bounds[i] <= (i ? bounds[i - 1] : 0)) return PF_ERR_ARG;     // strictly increasing, > 0
        if (fetch_ends && fetch_ends[i] < bounds[i]) return PF_ERR_ARG;
    }
    return haptag_bam_impl(ctx, K, bam, chrom, fetch_out, cov, truncated, n_bounds, bounds, fetch_ends);
}

// estimate_read_coverage_dirtyfast (blockjoin.c:951-1040) through the device
// fetch: the serial pass's records are, for a coordinate-sorted BAM, each
// contig's records in index order followed by the unplaced tail, so the pass
// is restated per contig -- whole-contig fetches (split into position pieces
// of bounded compressed size; a record counts in the piece its start falls
// in), the filters and 5 kb bins on the host from the gathered small fields.
// Its sequential quirks carry over: a truncated record ends the whole pass
// (its contig keeps the bins counted so far, later contigs 0), and unplaced
// reads at the end leave the last contig with reads at 0 (refID -1 when the
// loop ends).  Contigs without records stay 0.
// one contig of the device pass: *cov its estimate (0 without records),
// *stopped set by a truncated record (the serial pass ends there)
static int est_contig(pf_ctx_t *ctx, pf_bam_t *bam, int32_t t, uint64_t piece_bytes, int32_t *cov, bool *stopped,
                      bool *has_chunks) {
    *cov = 0;
    *stopped = false;
    const int64_t nc = pf_bam_query_chunks(bam, t, 0, INT64_MAX, nullptr, 0);
    if (nc < 0) return (int)nc;
    *has_chunks = nc > 0;
    if (nc == 0) return PF_OK;
    const uint32_t len = pf_bam_target_len(bam, t);
    int64_t step = 0;
    const uint64_t K = pf_bam_contig_pieces(bam, t, piece_bytes, &step);
    std::vector<uint64_t> bins(len / 5000, 0);
    for (uint64_t k = 0; k < K && !*stopped; k++) {
        const int64_t beg = (int64_t)k * step, end = k + 1 == K ? INT64_MAX : (int64_t)(k + 1) * step;
        pf_bam_dev_fetch_own F;
        const int rc = dev_fetch(ctx, bam, t, 1, &beg, &end, 0u, 0u, &F, [&](FetchOut &fo) -> int {
            const Small &S = *fo.S;
            for (uint64_t i = 0; i < fo.n; i++) {
                if (k && (int32_t)S.pos[i] < beg) continue;                 // counted in an earlier piece
                cov_add(bins, S, i);
            }
            return PF_OK;
        });
        if (rc) return rc;
        if (F.win_status[0] == PF_WIN_TRUNC) *stopped = true;
    }
    uint64_t tot = 0;
    for (uint64_t b : bins) tot += b;
    *cov = bins.empty() ? 0 : (int32_t)(tot / bins.size());
    return PF_OK;
}

extern "C" int pf_bam_estimate_contig_dev(pf_ctx_t *ctx, pf_bam_t *bam, int32_t tid, int32_t *cov, int32_t *truncated) {
    if (!ctx || !bam || !cov || !truncated || tid < 0 || tid >= pf_bam_n_targets(bam)) return PF_ERR_ARG;
    bool stopped = false, has = false;
    const int rc = est_contig(ctx, bam, tid, 0, cov, &stopped, &has);
    *truncated = stopped ? 1 : 0;
    return rc;
}

extern "C" int pf_bam_estimate_coverage_dev(pf_ctx_t *ctx, pf_bam_t *bam, int32_t *covs, int32_t n,
                                            uint64_t piece_bytes) {
    if (!ctx || !bam || !covs) return PF_ERR_ARG;
    const int32_t nr = pf_bam_n_targets(bam);
    if (n < nr) return PF_ERR_ARG;
    const int64_t n_unplaced = pf_bam_n_no_coor(bam);
    if (n_unplaced < 0) return pf_bam_estimate_coverage(bam, covs, n);
    for (int32_t i = 0; i < n; i++) covs[i] = 0;
    int32_t last = -1;
    bool stopped = false;
    for (int32_t t = 0; t < nr && !stopped; t++) {
        bool has = false;
        const int rc = est_contig(ctx, bam, t, piece_bytes, &covs[t], &stopped, &has);
        if (rc) return rc;
        if (has) last = t;
    }
    if (!stopped && n_unplaced > 0 && last >= 0) covs[last] = 0;
    return PF_OK;
}

// release the kept whole-contig arenas of a context (all contexts: NULL)
extern "C" void pf_fetch_cache_clear(pf_ctx_t *ctx) {
    std::vector<ArenaCache *> drop;
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        std::vector<ArenaCache *> keep;
        for (ArenaCache *c : g_cache) (ctx == nullptr || c->ctx == ctx ? drop : keep).push_back(c);
        g_cache.swap(keep);
    }
    for (ArenaCache *c : drop) {
        if (c->d_arena) arena_budget_give(pf_ctx_device((const pf_ctx *)c->ctx), c->arena + 512);
        (void)hipFree(c->d_arena);
        delete c;
    }
}

// keep the -u pre-pass's whole-contig arenas of a context for its window jobs
// (on), or stop and release them (off)
extern "C" void pf_fetch_cache_enable(pf_ctx_t *ctx, int on) {
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        auto it = std::find(g_keep_on.begin(), g_keep_on.end(), ctx);
        if (on && it == g_keep_on.end()) g_keep_on.push_back(ctx);
        if (!on && it != g_keep_on.end()) g_keep_on.erase(it);
    }
    if (!on) pf_fetch_cache_clear(ctx);
}
