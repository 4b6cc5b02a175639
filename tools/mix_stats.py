"""Per-window anatomy of the gap-mix bench batch (bench.py WORKLOADS["mix"]):
reads, sites, greedy iterations and the diagnostic build's K12 / K3 cycles
per window, the heaviest first -- what sets the step's tail.
usage: python tools/mix_stats.py [cache.npz] [n_windows] [workload]
With a cache path that does not exist the batch is generated, saved and the
script exits (generate outside the profiler / before the GPU call)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pomfret_amd._lib as L  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, load_aln, make_aln_batch, save_aln  # noqa: E402

cache = sys.argv[1] if len(sys.argv) > 1 else "-"
NW = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
wlname = sys.argv[3] if len(sys.argv) > 3 else "mix"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import WORKLOADS  # noqa: E402

wl = WORKLOADS[wlname]
if cache != "-" and os.path.exists(cache):
    aln = load_aln(cache)
else:
    aln = make_aln_batch(AlnSpec(n_windows=NW, coverage=wl["coverage"], gap=wl["gap"], seed=1000,
                                 gap_mix=wl["gap_mix"], skip_frac=wl["skip_frac"], nosite_frac=wl["nosite_frac"]),
                         workers=8)
    if cache != "-":
        save_aln(cache, aln)
        sys.exit(0)

prof = os.environ.get("PF_PROF", "1") == "1"
if prof:
    L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "libpomfret_amd_prof.so")
from pomfret_amd import Config, Context, LoadConfig  # noqa: E402

cov = wl["coverage"]
ctx = Context(0)
db = ctx.upload_aln(Config.from_coverage(cov, given=False), aln, LoadConfig())
for _ in range(3):
    out = db.run()
print("kernels", {k: round(v, 3) for k, v in ctx.kernel_times().items()})
st = db.stats()                                   # [W, 2, 8]: lookups inserts iters scanned summ nstrict R S
W = st.shape[0]
gap = (aln.win_end.astype(np.int64) - aln.win_start.astype(np.int64))
R = st[:, 0, 6].astype(np.int64)
S = np.maximum(st[:, 0, 7], st[:, 1, 7]).astype(np.int64)
it = st[:, :, 2].astype(np.int64)
print(f"windows {W}: reads p50 {np.median(R):.0f} max {R.max()}  sites p50 {np.median(S):.0f} max {S.max()}  "
      f"iters p50 {np.median(it):.0f} max {it.max()}  S>=8192: {(S >= 8192).sum()}  n_cand>64: "
      f"{0 if aln.win_n_cand is None else (aln.win_n_cand > 64).sum()}")
if prof:
    lib = L.lib()
    lib.pf_batch_prof.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    raw = np.zeros(W * 80, np.uint64)
    lib.pf_batch_prof(db.handle, raw.ctypes.data, raw.size)
    p3 = raw[:W * 64].reshape(W, 2, 32)
    k3c = (p3[:, :, :12].sum(axis=2) + p3[:, :, 16:24].sum(axis=2)).astype(float)
    k12p = raw[W * 64:].reshape(W, 16)[:, 1:7].astype(float)
    dz = raw[W * 64:].reshape(W, 16)[:, 0].astype(float)   # dense path: zero + atomics
    k12 = k12p.sum(axis=1)
    print("K12 cycles per window: p50 %.3g p90 %.3g max %.3g   K3 cycles per problem: p50 %.3g p90 %.3g max %.3g"
          % (np.median(k12), np.percentile(k12, 90), k12.max(), np.median(k3c), np.percentile(k3c, 90), k3c.max()))
    print("heaviest windows: w gap_kb reads sites iters(d0,d1) k12_cyc k3_cyc(d0,d1) decision")
    for w in np.argsort(-(k12 + k3c.max(axis=1)))[:16]:
        print(f"  {w:5d} {gap[w] / 1e3:7.1f} {R[w]:6d} {S[w]:6d} ({it[w, 0]},{it[w, 1]}) {k12[w]:.3g} "
              f"({k3c[w, 0]:.3g},{k3c[w, 1]:.3g}) {out.decision[w]}")
    names12 = ["T7+range", "sites", "revbuf", "dir arrays", "reservation", "methmers"]
    big = gap >= 150e3
    print("K12 phases, cycles: mean small (<150 kb) | mean big | heaviest window")
    hw = int(np.argmax(k12))
    print(f"  dense-path windows {(dz > 0).sum()}: zero+atomics cycles mean {dz[dz > 0].mean() if (dz > 0).any() else 0:.3g}, "
          f"heaviest {dz[hw]:.3g}")
    for j in range(6):
        print(f"    {names12[j]:12s} {k12p[~big, j].mean():10.0f} | {k12p[big, j].mean():10.0f} | {k12p[hw, j]:10.0f}")
    # cycles vs gap: the tail's shape
    for lo, hi in ((0, 20e3), (20e3, 50e3), (50e3, 150e3), (150e3, 600e3)):
        m = (gap >= lo) & (gap < hi)
        if m.any():
            print(f"  gap [{lo / 1e3:.0f},{hi / 1e3:.0f}) kb: {m.sum():4d} windows, reads {R[m].mean():.0f}, "
                  f"k12 {k12[m].mean():.3g}, k3 {k3c[m].max(axis=1).mean():.3g} cycles")
db.free()
ctx.close()
