"""Per-phase cycles of the greedy loop on the headline workload's heavy
problems, from the diagnostic (-DPF_K3_PROFILE) build (make -C
pomfret_amd/csrc prof): the bench's mix windows (seed 1000) -- the widest gaps
beside ordinary ones, as tests/test_headline_gpu.py -- at record level.

usage: python tools/k3_heavy_prof.py [n_ordinary | full]   (full: all 1024 windows of the mix)"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pomfret_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "libpomfret_amd_prof.so")
from pomfret_amd import Config, Context, LoadConfig  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, make_aln_batch  # noqa: E402

# stamp slots of k3_greedy_slim (K3_STAMP indices)
SLIM = {0: "init", 4: "range", 5: "collect", 6: "queue", 2: "prefetch+spans", 10: "fill", 3: "barrier B", 19: "pick", 20: "list shift",
        21: "insert", 8: "barrier X"}
SPEC = dict(n_windows=1024, coverage=60, gap=50_000, seed=1000, gap_mix=True, skip_frac=0.10, nosite_frac=0.05)
WIDE = [218, 422, 691, 580, 52, 884]
arg = sys.argv[1] if len(sys.argv) > 1 else "10"
wins = list(range(1024)) if arg == "full" else sorted(WIDE + list(range(int(arg))))
aln = make_aln_batch(AlnSpec(**SPEC), windows=wins, workers=16)
cfg, lcfg = Config.from_coverage(60, given=False), LoadConfig()
ctx = Context(0)
db = ctx.upload_aln(cfg, aln, lcfg)
db.run()
db.run()
kt = ctx.kernel_times()
print("greedy launch", db.k3_budget())
W = aln.n_windows
lib = L.lib()
lib.pf_batch_prof.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
raw = np.zeros(W * 80, np.uint64)
lib.pf_batch_prof(db.handle, raw.ctypes.data, raw.size)
prof = raw[:W * 64].reshape(W, 2, 32).astype(float)
st = db.stats()
heavy = {int(p) for p in db.heavy_problems()}
print(f"kernels {kt}")
print(f"heavy problems {sorted(heavy)}")
for label, sel in (("heavy", [p for p in range(2 * W) if p in heavy]),
                   ("main", [p for p in range(2 * W) if p not in heavy])):
    if not sel:
        continue
    it = sum(float(st[p >> 1, p & 1, 2]) for p in sel)
    tot = {k: sum(prof[p >> 1, p & 1, k] for p in sel) for k in SLIM}
    allc = sum(tot.values())
    print(f"{label}: {len(sel)} problems, {it:.0f} iterations, {allc / max(it, 1):.0f} cycles/iter")
    for k, n in SLIM.items():
        print(f"  {n:14s} {tot[k] / max(allc, 1) * 100:5.1f}%  {tot[k] / max(it, 1):8.0f} cyc/iter")
    print("  per problem (w,dir): reads, sites, iters, lookups/iter, methmers, Mcycles, path, KB")
    cyc = np.array([sum(prof[p >> 1, p & 1, k] for k in SLIM) for p in sel])
    print(f"  problem Mcycles: max {cyc.max() / 1e6:.2f}, p90 {np.percentile(cyc, 90) / 1e6:.2f}, "
          f"median {np.median(cyc) / 1e6:.2f}, sum {cyc.sum() / 1e9:.3f} G")
    paths = prof[[p >> 1 for p in sel], [p & 1 for p in sel], 29].astype(int)
    need = prof[[p >> 1 for p in sel], [p & 1 for p in sel], 31]
    nt = prof[[p >> 1 for p in sel], [p & 1 for p in sel], 30]
    print("  P2 path (1 LDS lists, 2 cache, 3 HBM lists, 4 body): " +
          ", ".join(f"{k}: {int((paths == k).sum())}" for k in (1, 2, 3, 4)))
    print(f"  LDS need of the slim layout taken: p50 {np.median(need) / 1024:.1f} KB, p90 "
          f"{np.percentile(need, 90) / 1024:.1f} KB, max {need.max() / 1024:.1f} KB; slots p50 {np.median(nt):.0f} "
          f"max {nt.max():.0f}")
    for p in sorted(sel, key=lambda p: -sum(prof[p >> 1, p & 1, k] for k in SLIM))[:8]:
        w, d = divmod(p, 2)
        print(f"    ({w},{d}) {st[w, d, 6]} {st[w, d, 7]} {st[w, d, 2]} {st[w, d, 0] / max(st[w, d, 2], 1):.0f} "
              f"{st[w, d, 4]} {sum(prof[w, d, k] for k in SLIM) / 1e6:.2f} {int(prof[w, d, 29])} "
              f"{prof[w, d, 31] / 1024:.1f}")
# the heaviest-first order against the measured per-problem cycles: list
# scheduling of those cycles over the resident slots (the main kernel's
# persistent grid) in three orders -- reads (k3_order today), methmers (the
# window's total over its reads), the measured cycles themselves (ideal)
if sel_all := [p for p in range(2 * W) if prof[p >> 1, p & 1, 29] > 0]:
    import heapq
    cyc_all = np.array([sum(prof[p >> 1, p & 1, k] for k in SLIM) for p in sel_all])
    reads_all = np.array([float(st[p >> 1, p & 1, 6]) for p in sel_all])
    mm_all = np.array([float(st[p >> 1, p & 1, 4]) for p in sel_all])
    slots = int(db.k3_budget()["resident"])
    def makespan(order):
        h = [0.0] * slots
        for i in order:
            t = heapq.heappop(h)
            heapq.heappush(h, t + cyc_all[i])
        return max(h)
    rw_ = np.diff(aln.win_rec_off.astype(np.int64))
    bases_w = np.add.reduceat(aln.l_qseq.astype(np.float64), aln.win_rec_off[:-1].astype(np.int64)) * (rw_ > 0)
    bases_all = np.array([bases_w[p >> 1] for p in sel_all])
    rec_all = np.array([float(rw_[p >> 1]) for p in sel_all])
    print(f"  corr(cycles, bases) {np.corrcoef(cyc_all, bases_all)[0, 1]:.3f}, corr(cycles, records) "
          f"{np.corrcoef(cyc_all, rec_all)[0, 1]:.3f}, corr(cycles, records^1.5) "
          f"{np.corrcoef(cyc_all, rec_all ** 1.5)[0, 1]:.3f}, corr(cycles, records x bases) "
          f"{np.corrcoef(cyc_all, rec_all * bases_all)[0, 1]:.3f}")
    for lab, key in (("reads", -reads_all), ("methmers", -mm_all), ("bases", -bases_all),
                     ("records x bases", -rec_all * bases_all), ("measured cycles", -cyc_all)):
        o = np.lexsort((np.arange(len(key)), key))
        print(f"  list schedule over {slots} slots by {lab:16s}: makespan {makespan(o) / 1e6:.2f} Mcycles")
    print(f"  corr(cycles, reads) {np.corrcoef(cyc_all, reads_all)[0, 1]:.3f}, corr(cycles, methmers) "
          f"{np.corrcoef(cyc_all, mm_all)[0, 1]:.3f}")
# concurrency over time from the problems' start/end (s_memrealtime, 100 MHz)
t0s = prof[:, :, 24].ravel()
t1s = prof[:, :, 25].ravel()
ok = (t0s > 0) & (t1s > t0s)
if ok.any():
    a0, a1 = t0s[ok], t1s[ok]
    base = a0.min()
    span = (a1.max() - base) / 100.0                     # microseconds
    grid = np.linspace(0, a1.max() - base, 41)
    conc = [int(((a0 - base <= g) & (a1 - base > g)).sum()) for g in grid]
    dur = (a1 - a0) / 100.0
    print(f"problems' span {span:.0f} us; duration us p50 {np.median(dur):.0f} max {dur.max():.0f}; "
          f"concurrency over time (41 samples): {conc}")
    print(f"  mean concurrency {np.mean(conc):.0f}; problem-us sum {dur.sum():.0f} -> mean "
          f"{dur.sum() / max(span, 1):.0f}")
    tr = prof[:, :, 26].ravel()[ok]
    if (tr > 0).any():
        pro = (a0 - tr)[tr > 0] / 100.0
        print(f"  prologue (k3_run start -> greedy init) us: p50 {np.median(pro):.1f} p90 {np.percentile(pro, 90):.1f} "
              f"max {pro.max():.1f}, sum {pro.sum():.0f} = {pro.sum() / dur.sum() * 100:.1f}% of the greedy loops' sum")
# the candidate-cache layout's LDS need against the window's reads (all problems)
allp = [(int(st[p >> 1, p & 1, 6]), prof[p >> 1, p & 1, 31] / 1024, sum(prof[p >> 1, p & 1, k] for k in SLIM) / 1e6)
        for p in range(2 * W) if prof[p >> 1, p & 1, 31] > 0]
if allp:
    a = np.array(allp)
    print("cache-layout need by reads (R bin: n, need p50 / p90 / max KB, Mcycles p50 / max):")
    for lo, hi in ((0, 300), (300, 450), (450, 600), (600, 800), (800, 1000), (1000, 1200), (1200, 5000)):
        sel = (a[:, 0] >= lo) & (a[:, 0] < hi)
        if sel.any():
            print(f"  [{lo},{hi}): {sel.sum():4d}  {np.median(a[sel, 1]):5.1f} / {np.percentile(a[sel, 1], 90):5.1f} / "
                  f"{a[sel, 1].max():5.1f}   {np.median(a[sel, 2]):.2f} / {a[sel, 2].max():.2f}")
    big = sorted(range(2 * W), key=lambda p: -prof[p >> 1, p & 1, 31])[:8]
    print("  largest needs (w,dir): reads sites slots need KB = cache KB + rest KB")
    for p in big:
        w, d = divmod(p, 2)
        print(f"    ({w},{d}) {st[w, d, 6]} {st[w, d, 7]} {prof[w, d, 30]:.0f} {prof[w, d, 31] / 1024:.1f} = "
              f"{prof[w, d, 27] / 1024:.1f} + {(prof[w, d, 31] - prof[w, d, 27]) / 1024:.1f}")
    for b in (32, 34, 36, 40, 44, 48):
        print(f"  need > {b} KB: {(a[:, 1] > b).sum()} problems, min reads among them "
              f"{int(a[a[:, 1] > b, 0].min()) if (a[:, 1] > b).any() else '-'}")
# K12 phases (K12_STAMP, cycles) per window: mean, the slowest window, and the
# kernel's window-cycles against its time (how many windows run at once)
k12 = raw[W * 64:].reshape(W, 16).astype(float)
names12 = ["-", "T7+range", "sites", "revbuf", "dir arrays", "reservation", "methmers"]
tot12 = k12[:, 1:7].sum(axis=1)
mx = int(tot12.argmax())
print(f"K12 phases, cycles: mean over windows | slowest window ({mx}: {int(st[mx, 0, 6])} reads, "
      f"{int(st[mx, 0, 7])} sites, gap {int(aln.win_end[mx]) - int(aln.win_start[mx])})")
for j in range(1, 7):
    print(f"  {names12[j]:12s} {k12[:, j].mean():10.0f} | {k12[mx, j]:10.0f}")
print(f"  window cycles: sum {tot12.sum() / 1e9:.3f} G, max {tot12.max() / 1e6:.2f} M, p90 "
      f"{np.percentile(tot12, 90) / 1e6:.2f} M, median {np.median(tot12) / 1e6:.2f} M")
kt12 = kt.get("pf_k12_sites_methmers", 0.0)
if kt12:
    print(f"  K12 {kt12:.3f} ms; sum of window cycles / (ms x 2.4 GHz) = "
          f"{tot12.sum() / (kt12 * 1e-3 * 2.4e9):.0f} windows at once on average (256 CUs)")
# the sites phase by path: k12[:, 0] packs the dense path's cycles (0: the fast
# path), its repeated positions (bits 32-51), the span in KiB (52-62) and
# whether the span fit the bitmap (63)
d0 = raw[W * 64:].reshape(W, 16)[:, 0].astype(np.uint64)
dense = d0 > 0
k12[:, 0] = (d0 & np.uint64(0xFFFFFFFF)).astype(float)
if dense.any():
    rep = ((d0 >> np.uint64(32)) & np.uint64(0xFFFFF)).astype(np.int64)[dense]
    spk = ((d0 >> np.uint64(52)) & np.uint64(0x7FF)).astype(np.int64)[dense]
    inr = (d0 >> np.uint64(63)).astype(bool)[dense]
    print(f"  dense windows: {int(inr.sum())} within the bitmap's span (repeated positions p50 "
          f"{int(np.median(rep[inr])) if inr.any() else 0}, min {int(rep[inr].min()) if inr.any() else 0}), "
          f"{int((~inr).sum())} beyond it (span KiB p50 {int(np.median(spk[~inr])) if (~inr).any() else 0}, "
          f"min {int(spk[~inr].min()) if (~inr).any() else 0}, max {int(spk[~inr].max()) if (~inr).any() else 0})")
rw = np.diff(aln.win_rec_off.astype(np.int64))
for lab, sel in (("fast path", ~dense), ("dense path", dense)):
    if sel.any():
        print(f"  sites phase, {lab}: {int(sel.sum())} windows, cycles mean {k12[sel, 2].mean():.0f} "
              f"p50 {np.median(k12[sel, 2]):.0f} max {k12[sel, 2].max():.0f}; share of all sites cycles "
              f"{k12[sel, 2].sum() / k12[:, 2].sum():.2f}; records p50 {np.median(rw[sel]):.0f}; "
              f"methmers phase mean {k12[sel, 6].mean():.0f}")
# sites-phase cycles per record (fast path): how they scale
if (~dense).any():
    cpr = k12[~dense, 2] / np.maximum(rw[~dense], 1)
    print(f"  fast-path sites cycles per record: p10 {np.percentile(cpr, 10):.0f} p50 {np.median(cpr):.0f} "
          f"p90 {np.percentile(cpr, 90):.0f}")
k2n = ["lb + ranges", "chars", "entries", "emission", "calls: flags+sites", "core tails", "loop back-edge"]
print("  K12 methmer phase, wave 0, cycles summed over its reads: mean over windows")
for j in range(7):
    print(f"    {k2n[j]:18s} {k12[:, 8 + j].mean():10.0f}")
db.free()
ctx.close()
