"""The bench's end-to-end leg alone (BAM file -> decisions through the device
fetch), for rocprofv3 kernel traces of the ingest kernels (pf_inflate,
pf_bgzf_crc, pf_chain, pf_recdec, pf_select, pf_gather_*) next to K0..K3.
usage: python tools/e2e_once.py <n_windows> <reps> <bam path: written when absent>"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
from pomfret_amd import Config, LoadConfig  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, make_aln_batch  # noqa: E402

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
path = sys.argv[3] if len(sys.argv) > 3 else "/tmp/pf_e2e.bam"
aln = make_aln_batch(AlnSpec(n_windows=nw, coverage=60, gap=50_000, seed=1000), workers=16)
if not os.path.exists(path):
    import _bamio
    recs = _bamio.records_from_aln(aln, qual=True)
    _bamio.write_bam(path, [("chrS", 2_000_000_000)], recs, workers=16, level=6)
    if reps == 0:
        sys.exit(0)
from pomfret_amd import Context  # noqa: E402
from pomfret_amd.bam import BamFile  # noqa: E402
ctx = Context(0)
cfg = Config.from_coverage(60, given=False)
with BamFile(path) as b:
    for _ in range(reps):
        t = time.perf_counter()
        db, qn, info = b.fetch_windows_device(ctx, cfg, "chrS", aln.win_start, aln.win_end, LoadConfig())
        out = db.run()
        db.free()
        ms = {k: round(v, 2) for k, v in info.items() if k.startswith("ms_")}
        print(f"{(time.perf_counter() - t) * 1e3:.1f} ms, {int(out.win_n_reads.sum())} reads, {ms}", flush=True)
