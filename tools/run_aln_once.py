"""One record-level batch of the bench workload (bench.py WORKLOAD: 1024
windows at 60x by default), uploaded and run a few times: the target of
rocprofv3 kernel-trace / PMC passes over K0..K3.
usage: python tools/run_aln_once.py [n_windows] [runs] [cache.npz] [coverage] [workload]
(workload: a bench.py WORKLOADS key, default bench.WORKLOAD)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pomfret_amd import Config, Context, LoadConfig  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, load_aln, make_aln_batch, save_aln  # noqa: E402

# argv: n_windows runs [cache.npz] [coverage]; with a cache path the batch is
# generated once (in worker processes, outside any profiler) and loaded
# afterwards.  Same seed as bench.py's rank 0 (strong scaling, N=1).
nw = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cache = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "-" else None
cov = int(sys.argv[4]) if len(sys.argv) > 4 else 60
from bench import WORKLOAD, WORKLOADS  # noqa: E402
wl = WORKLOADS[sys.argv[5]] if len(sys.argv) > 5 else WORKLOAD
if cache and os.path.exists(cache):
    aln = load_aln(cache)
else:
    aln = make_aln_batch(AlnSpec(n_windows=nw, coverage=cov, seed=1000, gap=wl["gap"], gap_mix=wl["gap_mix"],
                                 skip_frac=wl["skip_frac"], nosite_frac=wl["nosite_frac"]),
                         workers=int(os.environ.get("PF_SYNTH_WORKERS", "0")))
    if cache:
        save_aln(cache, aln)
        sys.exit(0)
ctx = Context(0)
db = ctx.upload_aln(Config.from_coverage(cov, given=False), aln, LoadConfig())
for _ in range(runs):
    db.run()
print(ctx.kernel_times())
db.free()
ctx.close()
