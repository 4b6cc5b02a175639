"""Run the bench workload a few times (profiling target for rocprofv3 --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pomfret_amd import Config, Context  # noqa: E402
from pomfret_amd.synth import SynthSpec, make_batch  # noqa: E402

cov = int(sys.argv[1]) if len(sys.argv) > 1 else 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = Config.from_coverage(cov, given=False)
b = make_batch(SynthSpec(n_windows=256, coverage=cov, gap=50_000, seed=1000))   # bench.py rank 0
ctx = Context(0)
db = ctx.upload(cfg, b)
for _ in range(reps):
    db.run()
print(ctx.kernel_times())
db.free()
ctx.close()
