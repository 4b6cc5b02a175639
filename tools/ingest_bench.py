"""Host ingest throughput (f1): write a synthetic BAM of n windows of the
bench workload (tests/_bamio.py writer, zlib level 1), then time
pf_bam_fetch_windows over all windows with 1 and N threads.
usage: python tools/ingest_bench.py [n_windows] [threads] [workdir]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))

import _bamio  # noqa: E402
from pomfret_amd.bam import BamFile  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, make_aln_batch  # noqa: E402

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 32
th = int(sys.argv[2]) if len(sys.argv) > 2 else 8
wd = sys.argv[3] if len(sys.argv) > 3 else "/tmp"
aln = make_aln_batch(AlnSpec(n_windows=nw, coverage=30, seed=1000))
recs = _bamio.records_from_aln(aln)
path = os.path.join(wd, "ingest.bam")
t = time.perf_counter()
_orig = _bamio.zlib.compressobj
_bamio.zlib.compressobj = lambda lvl, *a: _orig(1, *a)
_bamio.write_bam(path, [("chrS", 2_000_000_000)], recs)
print(f"wrote {len(recs)} records, {os.path.getsize(path) / 1e6:.0f} MB compressed, "
      f"{aln.nbytes() / 1e6:.0f} MB of record fields in {time.perf_counter() - t:.1f}s", flush=True)
with BamFile(path) as b:
    for n in (1, th):
        t = time.perf_counter()
        got, qn, _ = b.fetch_windows("chrS", aln.win_start, aln.win_end, threads=n)
        dt = time.perf_counter() - t
        print(f"threads={n}: {got.n_recs} records in {dt:.2f}s = {got.n_recs / dt:.0f} records/s, "
              f"{got.nbytes() / dt / 1e6:.0f} MB/s of record fields", flush=True)
