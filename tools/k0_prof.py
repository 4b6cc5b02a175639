"""Phase breakdown of the K0 loader from the diagnostic (-DPF_K0_PROFILE) build,
plus the K12 phases of the same record-level batch (run on the GPU box)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pomfret_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "libpomfret_amd_prof.so")
from pomfret_amd import Config, Context, LoadConfig  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, make_aln_batch  # noqa: E402

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cov = int(sys.argv[2]) if len(sys.argv) > 2 else 30
aln = make_aln_batch(AlnSpec(n_windows=nw, coverage=cov, seed=1000))
cfg = Config.from_coverage(cov, given=False)
ctx = Context(0)
db = ctx.upload_aln(cfg, aln, LoadConfig())
lib = L.lib()
before = np.zeros(16, np.uint64)
lib.pf_batch_load_counters(db.handle, before.ctypes.data, 16)
db.run()
after = np.zeros(16, np.uint64)
lib.pf_batch_load_counters(db.handle, after.ctypes.data, 16)
ph = (after - before)[8:12].astype(float)
R = db.n_reads
print(f"records {aln.n_recs} reads {R} kernels {ctx.kernel_times()}")
for n, v in zip(["MM stage+parse", "SEQ pass", "CIGAR walk+emit", "sort+endpos"], ph):
    print(f"  {n:18s} {v / R:10.0f} cyc/read  {v / ph.sum() * 100:5.1f}%")
lib.pf_batch_prof.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
raw = np.zeros(nw * 80, np.uint64)
lib.pf_batch_prof(db.handle, raw.ctypes.data, raw.size)
k12 = raw[nw * 64:].reshape(nw, 16).astype(float)
names12 = ["-", "T7+range", "sites", "revbuf", "dir arrays", "reservation", "methmers"]
mx = k12[:, 1:7].sum(axis=1).argmax()
print("  K12 phases, cycles: mean over windows | slowest window")
for j in range(1, 7):
    print(f"    {names12[j]:12s} {k12[:, j].mean():10.0f} | {k12[mx, j]:10.0f}")
# K3: per-(window, dir) greedy cycles of the same batch
prof = raw[:nw * 64].reshape(nw, 2, 32)
st = db.stats()
per = (prof[:, :, :12].sum(axis=2) + prof[:, :, 16:24].sum(axis=2)).astype(float).ravel()
it = st[:, :, 2].astype(float).ravel()
q = np.percentile(per, [50, 90, 99, 100])
print(f"  K3 problem cycles p50 {q[0]:.3g} p90 {q[1]:.3g} p99 {q[2]:.3g} max {q[3]:.3g}; "
      f"iters p50 {np.median(it):.0f} max {it.max():.0f}")
print("  K3 top problems (w,dir): cycles, iters, reads, sites, init cycles")
for i in np.argsort(per)[::-1][:6]:
    w, d = divmod(int(i), 2)
    print(f"    ({w},{d}) {per[i]:.3g} {it[i]:.0f} {st[w, d, 6]} {st[w, d, 7]} {float(prof[w, d, 0]):.3g}")
