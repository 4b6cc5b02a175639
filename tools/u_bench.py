"""--bam-is-untagged (-u) pre-pass benchmark (BASELINE configs[3] path, one
contig): synthetic SUP-like reads with CIGAR / MD:Z / 4-bit SEQ against
phased het variants every ~1 kb, tagged by pf_haptag_reads.

Reports the one-shot C-ABI rate (host SoA in, tags out: includes H2D), the
kernel-only rate from HIP events, the kernel's algorithmic bytes / time
(4 n_cigar + (l_MD + 1) + n_X + n_I_bases + 16 V_known_in_span
+ 1 per read) and the CPU oracle (single thread, the reference runs this pass
serially per contig) on the same reads.  Prints one JSON line.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pomfret_amd import Context  # noqa: E402
from pomfret_amd.synth_u import USpec, make_u_batch  # noqa: E402


def algo_bytes(known, reads):
    n_cig = len(reads.cigar)
    l_md = len(reads.md) + reads.n_reads
    kp = np.asarray(known.pos, np.int64)
    lo = np.searchsorted(kp, np.asarray(reads.start, np.int64))
    hi = np.searchsorted(kp, np.asarray(reads.end, np.int64))
    v_span = int((hi - lo).sum())
    md = bytes(np.asarray(reads.md, np.uint8))
    n_x = sum(md.count(c) for c in (b"A", b"C", b"G", b"T"))
    ins = int(sum((c >> 4) for c in np.asarray(reads.cigar, np.uint32) if (c & 0xf) == 1))
    return 4 * n_cig + l_md + n_x + ins + 16 * v_span + reads.n_reads


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16000
    spec = USpec(ref_len=4_000_000, n_reads=n, mean_len=12000, seed=11)
    t = time.time()
    known, reads, truth = make_u_batch(spec)
    gen_s = time.time() - t
    ctx = Context(0)
    hp = ctx.haptag_reads(known, reads)
    reps = 5
    t = time.perf_counter()
    kms = []
    for _ in range(reps):
        hp = ctx.haptag_reads(known, reads)
        kt = ctx.kernel_times()
        kms.append(kt.get("pf_k4_haptag", kt.get("pf_k4_thread", float("nan"))))
    wall = (time.perf_counter() - t) / reps
    kms = float(np.mean(kms))
    import oracle
    t = time.perf_counter()
    ref = oracle.haptag_reads(known, reads)
    cpu = time.perf_counter() - t
    assert np.array_equal(ref, hp), "parity"
    ab = algo_bytes(known, reads)
    print(json.dumps({
        "metric": "-u reads haplotagged/s", "reads": reads.n_reads, "known_variants": len(known.pos),
        "one_shot_reads_per_s": round(reads.n_reads / wall, 1), "one_shot_ms": round(wall * 1e3, 3),
        "kernel_ms": round(kms, 4), "kernel_reads_per_s": round(reads.n_reads / (kms * 1e-3), 1),
        "kernel_algo_bytes": ab, "kernel_GBps": round(ab / (kms * 1e-3) / 1e9, 2),
        "cpu_oracle_reads_per_s_1thread": round(reads.n_reads / cpu, 1),
        "truth_agreement": float((hp == truth).mean()), "gen_s": round(gen_s, 1)}))
    ctx.close()


if __name__ == "__main__":
    main()
