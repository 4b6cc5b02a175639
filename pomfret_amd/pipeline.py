"""`pomfret methphase` end to end with the GPU worker, host side in C:

    f3  pf_vcf_gaps           phase-block gaps of the phased VCF
                              (load_intervals_from_file + merge_close_intervals,
                              blockjoin.c:4442-4523)
    f1  pf_bam_fetch_windows  every gap's records, as load_reads_given_interval
                              fetches them (1053-1076)
    GPU pf_batch_upload_aln + pf_methphase_run per contig: K0 loader, K12, K3
                              (the kt_for worker, 4340-4426)
    f2  pf_phase_blocks, pf_write_gtf / _tsv / _vcf
                              (lift_decisions ... output_modify_vcf, 4685-4717)

The first-wins qname -> hp table of joined windows (4408-4423) is returned
for callers that write tags.  The dropped-interval rescue of the VCF writer
(recover_variant_phase_in_dropped_intervals, 2618-2694) needs a read pass
this pipeline does not make yet, so dropped intervals keep their sites as
the VCF writer leaves them without a rescue map.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from ._lib import Blocks, Context, Gaps
from .abi import Config, LoadConfig
from .bam import READBACK, BamFile


def methphase_files(bam_path: str, vcf_path: str, out_prefix: Optional[str], cfg: Config,
                    lcfg: Optional[LoadConfig] = None, device: int = 0, threads: int = 8,
                    ctx: Optional[Context] = None) -> Dict:
    """Run methphase over every gap of vcf_path with the reads of bam_path.
    Writes out_prefix + .mp.gtf / .mp.tsv / .mp.vcf unless out_prefix is None.
    Returns dict(decision=int8[n_gaps], contigs=[...], qname_hp={qname: hp})."""
    lcfg = lcfg or LoadConfig()
    gaps = Gaps(vcf_path, READBACK)
    own = ctx is None
    ctx = ctx or Context(device)
    decision = []
    qname_hp: Dict[str, int] = {}
    contigs = gaps.contigs()
    try:
        with BamFile(bam_path) as bam:
            for c in contigs:
                g = c["gaps"]
                if not g:
                    continue
                if bam.tid(c["name"]) < 0:
                    decision.extend([-1] * len(g))
                    continue
                ws = np.array([a for a, _ in g], np.uint32)
                we = np.array([b for _, b in g], np.uint32)
                aln, qn, _ = bam.fetch_windows(c["name"], ws, we, readback=READBACK, threads=threads)
                db = ctx.upload_aln(cfg, aln, lcfg)
                try:
                    out = db.run()
                    rec_of_read = db.read_recs()
                finally:
                    db.free()
                dec = np.asarray(out.decision, np.int8)
                decision.extend(dec.tolist())
                # reads -> windows: reads are the kept records in record order
                wro = np.searchsorted(rec_of_read, aln.win_rec_off.astype(np.int64))
                for w in range(len(g)):
                    if dec[w] < 0:
                        continue
                    for i in range(wro[w], wro[w + 1]):
                        q = qn[int(rec_of_read[i])]
                        if q not in qname_hp:               # first wins (4414-4421)
                            qname_hp[q] = int(out.read_hp[i])
        blocks = Blocks(gaps, np.asarray(decision, np.int8))
        if out_prefix is not None:
            blocks.write_gtf(out_prefix + ".mp.gtf")
            blocks.write_tsv(out_prefix + ".mp.tsv")
            blocks.write_vcf(vcf_path, out_prefix + ".mp.vcf")
        res = dict(decision=np.asarray(decision, np.int8), contigs=blocks.contigs(), qname_hp=qname_hp)
        blocks.close()
        return res
    finally:
        gaps.close()
        if own:
            ctx.close()
