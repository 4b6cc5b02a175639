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
SLIM = {0: "init", 2: "upkeep+spans", 10: "fill", 3: "barrier B", 19: "pick", 20: "list shift",
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
    print("  per problem (w,dir): reads, sites, iters, lookups/iter, methmers, Mcycles")
    cyc = np.array([sum(prof[p >> 1, p & 1, k] for k in SLIM) for p in sel])
    print(f"  problem Mcycles: max {cyc.max() / 1e6:.2f}, p90 {np.percentile(cyc, 90) / 1e6:.2f}, "
          f"median {np.median(cyc) / 1e6:.2f}, sum {cyc.sum() / 1e9:.3f} G")
    for p in sorted(sel, key=lambda p: -sum(prof[p >> 1, p & 1, k] for k in SLIM))[:8]:
        w, d = divmod(p, 2)
        print(f"    ({w},{d}) {st[w, d, 6]} {st[w, d, 7]} {st[w, d, 2]} {st[w, d, 0] / max(st[w, d, 2], 1):.0f} "
              f"{st[w, d, 4]} {sum(prof[w, d, k] for k in SLIM) / 1e6:.2f}")
db.free()
ctx.close()
