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

With untagged=True (`--bam-is-untagged`, -u) every contig's reads are first
haplotagged on the GPU from the VCF's phased variants (pf_vcf_known_vars +
pf_bam_fetch_contig_reads + pf_haptag_reads, the pre-pass of 1841-1898 with
its first-wins qname table) and those tags replace the BAM's HP in the
loader (1114-1122: a qname missing from the table is unphased).

The first-wins qname -> hp table of joined windows (4408-4423, merged across
contigs in contig order, 4572-4590) is returned for callers that write tags,
and drives the VCF writer's rescue of sites in dropped intervals
(recover_variant_phase_in_dropped_intervals, 2618-2694: pf_rescue_dropped
over the BAM).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from ._lib import Blocks, Context, Gaps
from .abi import Config, LoadConfig
from .bam import READBACK, BamFile, rescue_dropped, vcf_known_vars


def methphase_files(bam_path: str, vcf_path: str, out_prefix: Optional[str], cfg: Optional[Config],
                    lcfg: Optional[LoadConfig] = None, device: int = 0, threads: int = 8,
                    ctx: Optional[Context] = None, untagged: bool = False, tsv: bool = False) -> Dict:
    """Run methphase over every gap of vcf_path with the reads of bam_path.
    Writes out_prefix + .mp.gtf / .mp.vcf (and .mp.tsv with tsv=True, the
    reference's --tsv) unless out_prefix is None.
    cfg None: no -c, the per-contig parameters come from the BAM's coverage
    estimate (estimate_read_coverage_dirtyfast + 4358-4390).
    Returns dict(decision=int8[n_gaps], contigs=[...], qname_hp={qname: hp})."""
    lcfg = lcfg or LoadConfig()
    gaps = Gaps(vcf_path, READBACK)
    own = ctx is None
    ctx = ctx or Context(device)
    decision = []
    qname_hp: Dict[str, int] = {}
    raw_hp: Dict[str, int] = {}
    contigs = gaps.contigs()
    try:
        with BamFile(bam_path) as bam:
            est = bam.estimate_coverage() if cfg is None else None
            if untagged:                         # the pre-pass tags every contig first (2069-2080)
                for c in contigs:
                    if bam.tid(c["name"]) >= 0:
                        for q, h in _pre_haplotag(ctx, bam, vcf_path, c["name"]).items():
                            raw_hp.setdefault(q, h)
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
                if untagged:
                    aln.hp = np.array([raw_hp.get(q, 254) for q in qn], np.uint8)
                ccfg = cfg if cfg is not None else Config.from_coverage(est[bam.tid(c["name"])], given=False)
                db = ctx.upload_aln(ccfg, aln, lcfg)
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
            if tsv:
                blocks.write_tsv(out_prefix + ".mp.tsv")
            rescue = []
            with BamFile(bam_path) as bam:
                for c in contigs:
                    if not c["dropped"] or bam.tid(c["name"]) < 0:
                        rescue.append({})
                        continue
                    rescue.append(rescue_dropped(bam, c["name"], c["dropped"], vcf_known_vars(vcf_path, c["name"]),
                                                 qname_hp, raw_hp if untagged else None))
            blocks.write_vcf(vcf_path, out_prefix + ".mp.vcf", rescue=rescue)
        res = dict(decision=np.asarray(decision, np.int8), contigs=blocks.contigs(), qname_hp=qname_hp)
        blocks.close()
        return res
    finally:
        gaps.close()
        if own:
            ctx.close()


def _pre_haplotag(ctx: Context, bam: BamFile, vcf_path: str, contig: str) -> Dict[str, int]:
    """pre_haplotagging_read_in_one_ref (1841-1898) on the GPU: qname -> hp,
    first wins."""
    known = vcf_known_vars(vcf_path, contig)
    table: Dict[str, int] = {}
    if len(known.pos) == 0:
        return table
    reads, qn, _ = bam.fetch_contig_reads(contig)
    if len(qn) == 0:
        return table
    hp = ctx.haptag_reads(known, reads)
    for q, h in zip(qn, hp.tolist()):
        if q not in table:
            table[q] = int(h)
    return table
