"""Quick GPU-vs-oracle comparison on synthetic windows (developer tool)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pomfret_amd import Config, Context  # noqa: E402
from pomfret_amd.synth import SynthSpec, make_batch  # noqa: E402
import oracle  # noqa: E402


def compare(cfg, b, tag):
    t = time.time()
    ref = oracle.methphase(cfg, b, n_threads=8)
    t_cpu = time.time() - t
    ctx = Context(0)
    db = ctx.upload(cfg, b)
    t = time.time()
    out = db.run()
    t_gpu = time.time() - t
    ok = True
    for name in ("decision", "win_n_sites", "dir_table", "dir_join", "read_hp", "dir_which_way"):
        a, g = getattr(ref, name), getattr(out, name)
        if not np.array_equal(a, g):
            ok = False
            bad = np.argwhere(a != g)
            print(f"[{tag}] MISMATCH {name}: {len(bad)} diffs, first {bad[:5].tolist()}")
            if name in ("win_n_sites", "decision"):
                print("  ref", a.ravel()[:16], "\n  gpu", g.ravel()[:16])
    p_ok = np.allclose(ref.dir_fisher_p, out.dir_fisher_p, rtol=1e-6, atol=0)
    print(f"[{tag}] W={b.n_windows} R={b.n_reads} parity={'OK' if ok and p_ok else 'FAIL'} "
          f"cpu8={t_cpu:.3f}s gpu={t_gpu:.4f}s kernels={ctx.kernel_times()} "
          f"dec={np.bincount(out.decision + 1, minlength=3).tolist()}")
    db.free()
    ctx.close()
    return ok and p_ok


if __name__ == "__main__" and "--timing" not in sys.argv:
    allok = True
    allok &= compare(Config.from_coverage(30, given=False), make_batch(SynthSpec(n_windows=16, coverage=30)), "30x")
    allok &= compare(Config.from_coverage(60, given=True), make_batch(SynthSpec(n_windows=16, coverage=60, seed=2)), "60x")
    allok &= compare(Config.from_coverage(30, given=False), make_batch(SynthSpec(n_windows=16, coverage=30, seed=3, gap_mix=True)), "mix")
    print("ALL_OK" if allok else "SOME_FAIL")


def timing(n_windows=256, cov=30, reps=5):
    cfg = Config.from_coverage(cov, given=False)
    b = make_batch(SynthSpec(n_windows=n_windows, coverage=cov, seed=11))
    ctx = Context(0)
    db = ctx.upload(cfg, b)
    out = db.run()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        db.run(out)
        ts.append(time.perf_counter() - t)
    st = db.stats()
    print(f"[timing W={n_windows} cov={cov}] R={b.n_reads} wall min={min(ts)*1e3:.3f} ms "
          f"reads/s={b.n_reads/min(ts):.3e} kernels={ctx.kernel_times()}")
    print("  stats sum (lookups, inserts, iters, scanned):", st.sum(axis=(0, 1)).tolist(),
          " max iters/problem:", int(st[:, :, 2].max()))
    db.free()
    ctx.close()


if __name__ == "__main__" and "--timing" in sys.argv:
    timing(256, 30)
    timing(256, 60)
