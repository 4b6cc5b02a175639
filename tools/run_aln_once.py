"""One record-level batch (BASELINE configs[1] shape), uploaded and run a few
times: the target of rocprofv3 kernel-trace / PMC passes over K0..K3.
usage: python tools/run_aln_once.py [n_windows] [runs]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pomfret_amd import Config, Context, LoadConfig  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, load_aln, make_aln_batch, save_aln  # noqa: E402

# argv: n_windows runs [cache.npz]; with a cache path the batch is generated
# once (in worker processes, outside any profiler) and loaded afterwards
nw = int(sys.argv[1]) if len(sys.argv) > 1 else 256
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cache = sys.argv[3] if len(sys.argv) > 3 else None
if cache and os.path.exists(cache):
    aln = load_aln(cache)
else:
    aln = make_aln_batch(AlnSpec(n_windows=nw, coverage=30, seed=1000))
    if cache:
        save_aln(cache, aln)
        sys.exit(0)
ctx = Context(0)
db = ctx.upload_aln(Config.from_coverage(30, given=False), aln, LoadConfig())
for _ in range(runs):
    db.run()
print(ctx.kernel_times())
db.free()
ctx.close()
