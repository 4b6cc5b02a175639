"""`pomfret methphase` end to end on the CPU oracle -- TEST INFRASTRUCTURE.

The same chain as the product's pipeline, with every compute step taken from
the oracle: gaps (oracle.vcf_gaps, blockjoin.c:4442-4523), the -u pre-pass
(oracle.haptag_reads over each contig's reads, 1841-1898, qname first-wins
1880-1889, merged over contigs first-wins), per window the loader + worker
(oracle.load_reads + oracle.methphase: 1043-1173, 4217-4335), the joined
windows' qname -> hp table (first wins in (contig, window) order,
4408-4423 / 4572-4590), the dropped-interval rescue (tests/test_bam.py's
restatement of 2618-2694) and the epilogue (oracle/epilogue.py: lift,
blocks, GTF/TSV/VCF, 2250-2988).  Records come from the product's BAM
reader, which tests/test_bam.py checks against the test-side writer."""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def methphase_files_oracle(bam_path, vcf_path, cfg, lcfg=None, untagged=False, recs_by_contig=None,
                           n_threads=8):
    """-> dict(decision, qname_hp, raw_hp, gtf, tsv, vcf, counts).  recs_by_contig
    ({contig: [Rec]} as written) feeds the rescue restatement."""
    import oracle
    from oracle import epilogue as ep
    from pomfret_amd import LoadConfig
    from pomfret_amd.bam import BamFile, vcf_known_vars
    from test_bam import _py_rescue

    lcfg = lcfg or LoadConfig()
    contigs = oracle.vcf_gaps(vcf_path)
    decision, qname_hp, raw_hp = [], {}, {}
    with BamFile(bam_path) as bam:
        if untagged:
            for c in contigs:
                if bam.tid(c["name"]) < 0:
                    continue
                kv = vcf_known_vars(vcf_path, c["name"])
                if len(kv.pos) == 0:
                    continue
                reads, qn, _ = bam.fetch_contig_reads(c["name"])
                if not qn:
                    continue
                hp = oracle.haptag_reads(kv, reads)
                tab = {}
                for q, h in zip(qn, hp.tolist()):
                    tab.setdefault(q, int(h))
                for q, h in tab.items():
                    raw_hp.setdefault(q, h)
        for c in contigs:
            g = c["gaps"]
            if not g:
                continue
            if bam.tid(c["name"]) < 0:
                decision += [-1] * len(g)
                continue
            ws = np.array([a for a, _ in g], np.uint32)
            we = np.array([b for _, b in g], np.uint32)
            aln, qn, _ = bam.fetch_windows(c["name"], ws, we)
            if untagged:
                aln.hp = np.array([raw_hp.get(q, 254) for q in qn], np.uint8)
            wb, rec_read = oracle.load_reads(lcfg, aln)
            res = oracle.methphase(cfg, wb, n_threads=n_threads)
            recs_of_read = np.flatnonzero(rec_read != 0xFFFFFFFF)
            dec = res.decision.astype(np.int8)
            decision += dec.tolist()
            ro = wb.win_read_off.astype(np.int64)
            for w in range(len(g)):
                if dec[w] < 0:
                    continue
                for i in range(ro[w], ro[w + 1]):
                    qname_hp.setdefault(qn[int(recs_of_read[i])], int(res.read_hp[i]))
    blocks = ep.phase_blocks(contigs, decision)
    rescue = []
    for c in contigs:
        if not c["dropped"] or recs_by_contig is None or c["name"] not in recs_by_contig:
            rescue.append({})
            continue
        kv = vcf_known_vars(vcf_path, c["name"])
        rescue.append(_py_rescue(recs_by_contig[c["name"]], kv.pos.tolist(), c["dropped"], qname_hp,
                                 raw_hp if untagged else None))
    vcf, counts = ep.vcf_bytes(vcf_path, contigs, blocks, rescue)
    return dict(decision=np.asarray(decision, np.int8), qname_hp=qname_hp, raw_hp=raw_hp,
                gtf=ep.gtf_text(contigs, blocks), tsv=ep.tsv_text(contigs, blocks), vcf=vcf, counts=counts)
