"""Phase breakdown of the greedy kernel from the diagnostic (-DPF_K3_PROFILE) build."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pomfret_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "libpomfret_amd_prof.so")
from pomfret_amd import Config, Context  # noqa: E402
from pomfret_amd.synth import SynthSpec, make_batch  # noqa: E402

names = ["init", "setup", "publish", "barrierB", "fold(chunked)", "pick fallback", "winner fields", "tail:spans",
         "barrierA", "fields", "fill_rows", "groupsum",
         "upkeep:collect", "upkeep:next read", "pick:lcode", "pick_exact",
         "tail:insert", "tail:hp/untag", "tail:shift", "tail:range update"]
NW = int(sys.argv[1]) if len(sys.argv) > 1 else 256
COVS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [30, 60]
for cov in COVS:
    cfg = Config.from_coverage(cov, given=False)
    b = make_batch(SynthSpec(n_windows=NW, coverage=cov, seed=11))
    ctx = Context(0)
    db = ctx.upload(cfg, b)
    db.run(); db.run()
    lib = L.lib()
    lib.pf_batch_prof.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    raw = np.zeros(NW * 80, np.uint64)
    lib.pf_batch_prof(db.handle, raw.ctypes.data, raw.size)
    prof = raw[:NW * 64].reshape(NW, 2, 32)
    k12 = raw[NW * 64:].reshape(NW, 16).astype(float)
    st = db.stats()
    cnt = prof[:, :, 12:16].sum(axis=(0, 1)).astype(float)
    tot = np.concatenate([prof[:, :, :12], prof[:, :, 16:24]], axis=2).sum(axis=(0, 1)).astype(float)
    iters = st[:, :, 2].sum()
    print(f"cov={cov} kernels={ctx.kernel_times()} iters={iters}")
    for n, v in zip(names, tot):
        print(f"  {n:18s} {v/tot.sum()*100:5.1f}%  {v/iters:8.0f} cyc/iter")
    per = (prof[:, :, :12].sum(axis=2) + prof[:, :, 16:24].sum(axis=2)).astype(float).ravel()
    it = st[:, :, 2].astype(float).ravel()
    top = np.argsort(per)[::-1][:6]
    print("  top problems (w,dir): cycles, iters, init cycles, reads, sites, lookups/iter, one_chunk")
    for i in top:
        w, d = divmod(int(i), 2)
        print(f"    ({w},{d}) {per[i]:.3g} {it[i]:.0f} {float(prof[w, d, 0]):.3g} {st[w, d, 6]} {st[w, d, 7]} "
              f"{st[w, d, 0] / max(it[i], 1):.0f} {prof[w, d, 15]}")
    ev = prof[:, :, 24:28].sum(axis=(0, 1)).astype(float)
    print(f"  loop back-edge (tail end -> loop top, wave 0): {prof[:, :, 28].sum() / iters:.0f} cyc/iter")
    print(f"  per iter: failed picks {ev[0]/iters:.3f}  collects {ev[1]/iters:.3f}  "
          f"collect rebuilds {ev[2]/iters:.3f}  queue refills {ev[3]/iters:.3f}")
    print(f"  median problem cycles {np.median(per):.3g}, mean {per.mean():.3g}, max {per.max():.3g}, "
          f"p90 {np.percentile(per, 90):.3g}")
    print(f"  per iter: lmax(chunked) {cnt[0]/iters:.1f}  nc(one-chunk) {cnt[1]/iters:.2f}  "
          f"picks needing the sequential fold {cnt[2]/iters*100:.2f}%")
    names12 = ["-", "T7+range", "sites", "revbuf", "dir arrays", "reservation", "methmers"]
    mx = k12.sum(axis=1).argmax()
    print("  K12 phases, cycles: mean over windows | slowest window")
    for j in range(1, 7):
        print(f"    {names12[j]:12s} {k12[:, j].mean():10.0f} | {k12[mx, j]:10.0f}")
    k2n = ["lb + ranges", "chars", "entries", "emission", "calls: flags+sites", "core tails",
           "loop back-edge"]
    print("  K12 methmer phase, wave 0, cycles summed over its reads: mean over windows")
    for j in range(7):
        print(f"    {k2n[j]:18s} {k12[:, 8 + j].mean():10.0f}")
    print(f"    {'loop end (moves)':18s} {k12[:, 7].mean():10.0f}")
    print(f"    {'prefetch issue':18s} {k12[:, 15].mean():10.0f}")
    db.free(); ctx.close()
