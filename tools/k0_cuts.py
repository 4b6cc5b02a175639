"""K0 phase costs as kernel-time differences: the same resident batch run
with PF_K0_DIAG = 4 (filters only), 2 (+ MM/ML), 3 (+ SEQ pass) and 0 (the
whole kernel).  Measurement only: the cut runs' results are invalid.
usage: python tools/k0_cuts.py [n_windows] [workload] [runs]"""
import os
import subprocess
import sys

if len(sys.argv) > 4:                               # child: one mode
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import WORKLOADS
    from pomfret_amd import Config, Context, LoadConfig
    from pomfret_amd.synth_aln import AlnSpec, load_aln
    aln = load_aln(sys.argv[4])
    ctx = Context(0)
    db = ctx.upload_aln(Config.from_coverage(60, given=False), aln, LoadConfig())
    acc = 0.0
    n = int(sys.argv[3])
    db.run()
    for _ in range(n):
        db.run()
        acc += ctx.kernel_times()["pf_k0_load"]
    print(f"{os.environ.get('PF_K0_DIAG', '0')} {acc / n:.4f}")
    sys.exit(0)

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
wl = sys.argv[2] if len(sys.argv) > 2 else "fixed50"
runs = sys.argv[3] if len(sys.argv) > 3 else "5"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import WORKLOADS  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, make_aln_batch, save_aln  # noqa: E402
w = WORKLOADS[wl]
path = "/tmp/k0cuts.npz"
save_aln(path, make_aln_batch(AlnSpec(n_windows=nw, coverage=w["coverage"], gap=w["gap"], seed=1000,
                                      gap_mix=w["gap_mix"], skip_frac=w["skip_frac"],
                                      nosite_frac=w["nosite_frac"]), workers=8))
res = {}
for mode in ("4", "2", "5", "3", "0"):
    env = dict(os.environ, PF_K0_DIAG=mode)
    out = subprocess.run([sys.executable, __file__, str(nw), wl, runs, path], env=env, capture_output=True,
                         text=True, timeout=300)
    if out.returncode:
        print(out.stderr[-2000:])
        sys.exit(out.returncode)
    m, t = out.stdout.split()[-2:]
    res[m] = float(t)
    print(f"PF_K0_DIAG={m}: K0 {float(t):.3f} ms", flush=True)
print(f"filters+launch {res['4']:.3f}  MM/ML {res['2'] - res['4']:.3f}  SEQ {res['3'] - res['2']:.3f} "
      f"(count+range {res['5'] - res['2']:.3f}, placement {res['3'] - res['5']:.3f})  "
      f"CIGAR+emit+end {res['0'] - res['3']:.3f} ms")
