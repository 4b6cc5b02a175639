"""Whole-genome-shaped synthetic BAM + phased VCF -- TEST / BENCH
INFRASTRUCTURE (never imported by the product).

BASELINE configs[3] is `pomfret methphase -u` without -c on a WGS BAM: many
contigs, thousands of phase-block gaps, every read untagged.  synth_aln's
windows are independent (each has its own reference and reads); here each
contig is one reference sequence with reads drawn uniformly over it, so
adjacent windows share reads, the -u pre-pass and the coverage pass see every
read of the contig, and the phase blocks come from a phased VCF:

* contig layout: phase blocks (log-uniform block_min..block_max, a
  short_block_frac of them shorter than READBACK so merge_close_intervals
  drops them, blockjoin.c:2190-2217) separated by gaps (log-uniform
  gap_min..gap_max); het SNVs at het_snv_rate inside the blocks only, one
  on each block's first and last base so insert_vcf_line's gap is exactly
  [last POS of a block, PS of the next] (1416-1418); a random phase
  orientation per block (the VCF's hap index = truth haplotype ^ orient);
* reference with CpGs only where planted, site classes, reads, CIGAR/SEQ/MD
  and MM/ML: synth_aln's read model (`_build_reads`), HP absent (-u);
* BAM: records in coordinate order, compressed in worker processes in chunks
  of consecutive reads (BGZF blocks of 0xFF00 bytes within a chunk), a BAI
  built as tests/_bamio.bai_bytes does; QUAL strings of nanopore-like
  entropy so the BGZF sizes are a real BAM's.

Everything is a pure function of the spec (seeded per contig and chunk).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from _bamio import (BLOCK, EOF_BLOCK, Rec, _deflate_block, aux_BC, aux_f, aux_i, aux_Z, bai_bytes,  # noqa: E402
                    bam_header, encode_record, endpos)

A_, C_, G_ = 0, 1, 2


@dataclass
class GenomeSpec:
    contigs: tuple = (("chr1", 30_000_000), ("chr2", 26_000_000), ("chr3", 22_000_000), ("chr4", 18_000_000))
    coverage: float = 60.0
    block_min: int = 50_000
    block_max: int = 100_000
    short_block_frac: float = 0.05
    gap_min: int = 5_000
    gap_max: int = 40_000
    lead: int = 100_000
    seed: int = 2025
    aln: object = None            # synth_aln.AlnSpec of the read model (default: -u, het SNVs 1/kb)
    qual: bool = True
    level: int = 6
    chunk_reads: int = 1000
    hp_tags: bool = False         # HP:i from the phase of the block a read starts in (pre-haplotagged BAM)

    def read_spec(self):
        from pomfret_amd.synth_aln import AlnSpec
        return self.aln or AlnSpec(het_snv_rate=0.001, untag_frac=0.0)


def _logu(rng, lo, hi):
    return int(np.exp(rng.uniform(np.log(lo), np.log(hi))))


def contig_layout(spec: GenomeSpec, ci: int) -> dict:
    """Reference, CpG sites, phase blocks, het SNVs and reads of contig ci."""
    from pomfret_amd.synth import _lognormal_params
    rs = spec.read_spec()
    name, L = spec.contigs[ci]
    rng = np.random.default_rng([spec.seed, ci, 1])
    ref = rng.integers(0, 4, L).astype(np.uint8)
    cg = np.flatnonzero((ref[:-1] == C_) & (ref[1:] == G_))
    ref[cg + 1] = A_
    cpg = np.unique(rng.integers(1, L - 3, size=rng.poisson(rs.cpg_rate * L)))
    cpg = cpg[np.concatenate([[True], np.diff(cpg) >= 2])]
    ref[cpg] = C_
    ref[cpg + 1] = G_
    cls = rng.random(cpg.shape[0])
    site_p = np.where(cls < 0.7, 0.95, 0.05)
    site_asm = cls >= 0.9
    site_hap = rng.integers(0, 2, cpg.shape[0])
    site_of = np.full(L, -1, np.int32)
    site_of[cpg] = np.arange(cpg.shape[0], dtype=np.int32)

    blocks = []
    pos = spec.lead
    while True:
        if rng.random() < spec.short_block_frac:
            bl = _logu(rng, 10_000, 50_000)
        else:
            bl = _logu(rng, spec.block_min, spec.block_max)
        if pos + bl + spec.lead > L:
            break
        blocks.append((pos, pos + bl))
        pos += bl + _logu(rng, spec.gap_min, spec.gap_max)
    blocks = np.array(blocks, np.int64).reshape(-1, 2)
    orient = rng.integers(0, 2, blocks.shape[0])

    is_cpg = np.zeros(L, bool)
    is_cpg[cpg] = True
    is_cpg[cpg + 1] = True
    snv_pos, snv_blk = [], []
    for b, (bs, be) in enumerate(blocks.tolist()):
        n = rng.poisson(rs.het_snv_rate * (be - bs))
        p = np.unique(rng.integers(bs + 1, be - 1, n))
        p = p[~is_cpg[p]]
        p = np.unique(np.concatenate([[bs, be - 1], p]))        # the block's ends stay, CpG or not
        snv_pos.append(p)
        snv_blk.append(np.full(p.shape[0], b))
    snv_pos = np.concatenate(snv_pos) if snv_pos else np.zeros(0, np.int64)
    snv_blk = np.concatenate(snv_blk) if snv_blk else np.zeros(0, np.int64)
    snv_ref = ref[snv_pos].copy()
    snv_alt = ((snv_ref + rng.integers(1, 4, snv_pos.shape[0])) % 4).astype(np.uint8)
    h_alt = rng.integers(0, 2, snv_pos.shape[0]).astype(np.int64)
    alt_of = np.full(L, -1, np.int16)
    halt_of = np.full(L, -1, np.int16)
    alt_of[snv_pos] = snv_alt
    halt_of[snv_pos] = h_alt

    rng2 = np.random.default_rng([spec.seed, ci, 2])
    mu, sig = _lognormal_params(rs.mean_len, rs.sd_len)
    n = int(spec.coverage * L / rs.mean_len)
    lens = np.clip(np.exp(rng2.normal(mu, sig, n)), rs.min_len, rs.max_len).astype(np.int64)
    starts = (rng2.random(n) * (L - lens - 2)).astype(np.int64) + 1
    o = np.argsort(starts, kind="stable")
    starts, lens = starts[o], lens[o]
    truth = rng2.integers(0, 2, n)
    strand = (rng2.random(n) < 0.5).astype(np.int64)
    return dict(name=name, L=L, ref=ref, site_of=site_of, site_p=site_p, site_asm=site_asm, site_hap=site_hap,
                blocks=blocks, orient=orient, snv=dict(pos=snv_pos, blk=snv_blk, ref=snv_ref, alt=snv_alt,
                                                       h_alt=h_alt, alt_of=alt_of, halt_of=halt_of),
                starts=starts, lens=lens, truth=truth, strand=strand)


_G = {}          # contig layouts, shared with the fork workers


def _chunk_job(args):
    """Records [r0, r1) of contig ci: encoded, BGZF-compressed in blocks of
    0xFF00 bytes.  -> (blocks, raw block lengths, per record (tid, pos, end,
    flag, start byte, end byte) within the chunk stream, Recs if keep)."""
    spec, ci, k, r0, r1, keep = args
    from pomfret_amd.synth_aln import _build_reads
    g = _G[ci]
    rs = spec.read_spec()
    rng = np.random.default_rng([spec.seed, ci, 3, k])
    sl = slice(r0, r1)
    out, flag, mapq, de = _build_reads(rs, rng, g["ref"], g["starts"][sl], g["lens"][sl], g["truth"][sl],
                                       g["strand"][sl], g["site_of"], g["site_p"], g["site_asm"], g["site_hap"],
                                       g["snv"])
    hp_of = None
    if spec.hp_tags:                                    # the VCF's hap index of the read's block: truth ^ orient
        st_ = g["starts"][sl]
        blk = np.searchsorted(g["blocks"][:, 0], st_, side="right") - 1
        inb = (blk >= 0) & (st_ < g["blocks"][np.maximum(blk, 0), 1])
        hp_of = np.where(inb, g["truth"][sl] ^ g["orient"][np.maximum(blk, 0)], 254)
        hp_of[np.random.default_rng([spec.seed, ci, 6, k]).random(r1 - r0) < 0.1] = 254
    qpool = None
    if spec.qual:
        qpool = np.random.default_rng([spec.seed, ci, 4, k]).normal(20, 6, 1 << 21).clip(2, 50) \
            .astype(np.uint8).tobytes()
        qoff = np.random.default_rng([spec.seed, ci, 5, k]).integers(0, 1 << 20, r1 - r0)
    stream = bytearray()
    ents, recs = [], []
    for i, r in enumerate(out):
        aux = b""
        if de[i] >= 0:
            aux += aux_f("de", float(de[i]))
        if r["mm"].shape[0]:
            aux += aux_Z("MM", r["mm"].tobytes().decode())
        if r["ml"].shape[0]:
            aux += aux_BC("ML", r["ml"])
        if "md" in r:
            aux += aux_Z("MD", r["md"])
        if spec.hp_tags and hp_of is not None and hp_of[i] != 254:
            aux += aux_i("HP", int(hp_of[i]) + 1)
        lq = int(r["l_qseq"])
        q = None
        if qpool is not None:
            o = int(qoff[i]) % max(1, len(qpool) - lq)
            q = qpool[o:o + lq]
        rec = Rec(tid=ci, pos=int(g["starts"][r0 + i]), qname=f"{g['name']}_{r0 + i}", flag=int(flag[i]),
                  mapq=int(mapq[i]), cigar=[int(x) for x in r["cigar"]], seq=r["seq"].tobytes(), l_seq=lq,
                  aux=aux, qual=q)
        b0 = len(stream)
        stream += encode_record(rec)
        ents.append((ci, rec.pos, endpos(rec.pos, rec.cigar, rec.flag), rec.flag, b0, len(stream)))
        if keep:
            recs.append(rec)
    blocks = [_deflate_block((bytes(stream[i:i + BLOCK]), spec.level)) for i in range(0, len(stream), BLOCK)]
    return blocks, len(stream), ents, recs


def write_genome(prefix: str, spec: GenomeSpec, workers: int = 8, keep_recs: bool = False) -> dict:
    """Write prefix.bam (+ .bai) and prefix.vcf.  -> dict(bam, vcf, refs,
    n_records, bam_bytes, n_blocks (phase blocks), n_snvs, recs_by_contig
    ({name: [Rec]} with keep_recs))."""
    import multiprocessing as mp
    refs = [(n, int(L)) for n, L in spec.contigs]
    _G.clear()
    for ci in range(len(refs)):
        _G[ci] = contig_layout(spec, ci)
    tasks = []
    for ci in range(len(refs)):
        n = _G[ci]["starts"].shape[0]
        for k, r0 in enumerate(range(0, n, spec.chunk_reads)):
            tasks.append((spec, ci, k, r0, min(n, r0 + spec.chunk_reads), keep_recs))
    bam = prefix + ".bam"
    entries = []
    recs_by = {n: [] for n, _ in refs}
    n_rec = 0
    with open(bam, "wb") as f:
        hb = _deflate_block((bam_header(refs), spec.level))
        f.write(hb)
        addr = len(hb)
        ctx = mp.get_context("fork")
        pool = ctx.Pool(workers) if workers > 1 else None
        try:
            it = pool.imap(_chunk_job, tasks, chunksize=1) if pool else map(_chunk_job, tasks)
            for blocks, total, ents, recs in it:
                baddr = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.int64) + addr
                nxt = int(baddr[-1])

                def voff(p):
                    if p == total:                     # the chunk's end: the next block's start
                        return nxt << 16
                    return (int(baddr[p // BLOCK]) << 16) | (p % BLOCK)

                for t, pos, end, flag, b0, b1 in ents:
                    entries.append((t, pos, end, flag, voff(b0), voff(b1)))
                for b in blocks:
                    f.write(b)
                addr = nxt
                n_rec += len(ents)
                if recs:
                    recs_by[refs[recs[0].tid][0]] += recs
        finally:
            if pool:
                pool.close()
                pool.join()
        f.write(EOF_BLOCK)
    with open(bam + ".bai", "wb") as f:
        f.write(bai_bytes(len(refs), entries))
    vcf = prefix + ".vcf"
    n_snv = write_genome_vcf(vcf, refs)
    res = dict(bam=bam, vcf=vcf, refs=refs, n_records=n_rec, bam_bytes=os.path.getsize(bam),
               n_blocks=int(sum(_G[c]["blocks"].shape[0] for c in _G)), n_snvs=n_snv)
    if keep_recs:
        res["recs_by_contig"] = recs_by
    _G.clear()
    return res


def write_genome_vcf(path: str, refs) -> int:
    """The phased VCF of the contig layouts in _G: every het SNV, GT a|b with
    ALT on the block's hap index h_alt ^ orient, PS = the block's first POS."""
    lines = ["##fileformat=VCFv4.2"] + [f"##contig=<ID={n},length={L}>" for n, L in refs] + [
        '##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype">',
        '##FORMAT=<ID=PS,Number=1,Type=Integer,Description="Phase set">',
        "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1"]
    n = 0
    for ci in range(len(refs)):
        g = _G[ci]
        s = g["snv"]
        ps_of = g["blocks"][:, 0] + 1
        v = s["h_alt"] ^ g["orient"][s["blk"]]
        for p, r, a, b, hv in zip(s["pos"].tolist(), s["ref"].tolist(), s["alt"].tolist(), s["blk"].tolist(),
                                  v.tolist()):
            gt = "0|1" if hv == 1 else "1|0"
            lines.append(f"{g['name']}\t{p + 1}\t.\t{'ACGT'[r]}\t{'ACGT'[a]}\t50\tPASS\t.\tGT:PS\t{gt}:{ps_of[b]}")
            n += 1
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return n


def small_spec(seed: int = 7) -> GenomeSpec:
    """A few-Mb genome of the same shape for GPU parity tests (half-length
    reads so the oracle pipeline finishes in seconds)."""
    from pomfret_amd.synth_aln import AlnSpec
    return GenomeSpec(contigs=(("chr1", 1_300_000), ("chr2", 900_000), ("chr3", 700_000), ("chr4", 500_000)),
                      coverage=40, block_min=40_000, block_max=90_000, short_block_frac=0.15,
                      gap_min=5_000, gap_max=40_000, lead=60_000, seed=seed, qual=False, level=1,
                      chunk_reads=400,
                      aln=AlnSpec(het_snv_rate=0.001, untag_frac=0.0, mean_len=15_000, sd_len=7_500,
                                  min_len=7_500, max_len=75_000))


def pieces_spec(seed: int = 5) -> GenomeSpec:
    """One 3 Mb contig whose phase blocks (250-400 kb) leave room between the
    windows' fetch regions (gap + 2 x 50 kb): the -u pre-pass's position
    pieces (forced small with PF_FETCH_PIECE_BYTES) get bounds between
    windows, so every window job is served by one kept piece arena."""
    from pomfret_amd.synth_aln import AlnSpec
    return GenomeSpec(contigs=(("chrP", 3_000_000),), coverage=30, block_min=250_000, block_max=400_000,
                      short_block_frac=0.0, gap_min=5_000, gap_max=40_000, lead=60_000, seed=seed, qual=False,
                      level=1, chunk_reads=400,
                      aln=AlnSpec(het_snv_rate=0.001, untag_frac=0.0, mean_len=15_000, sd_len=7_500,
                                  min_len=7_500, max_len=75_000))


def report_spec(seed: int = 11) -> GenomeSpec:
    """BASELINE configs[4]'s shape at test scale: a 200x pileup over one
    contig with pre-haplotagged reads, phase blocks of 40-90 kb (the report's
    chunk windows sample inside them) and half-length reads."""
    from pomfret_amd.synth_aln import AlnSpec
    return GenomeSpec(contigs=(("chr1", 560_000),), coverage=200, block_min=40_000, block_max=90_000,
                      short_block_frac=0.0, gap_min=5_000, gap_max=30_000, lead=60_000, seed=seed, qual=False,
                      level=1, chunk_reads=500, hp_tags=True,
                      aln=AlnSpec(het_snv_rate=0.001, untag_frac=0.0, mean_len=15_000, sd_len=7_500,
                                  min_len=7_500, max_len=60_000))
