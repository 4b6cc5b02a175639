"""BAM + VCF fixtures for the end-to-end tests (test infrastructure): the
records of synth_aln windows written by the test-side BAM writer
(tests/_bamio.py) with a phased VCF whose phase-block gaps are the
windows."""
import os

import numpy as np

from tests._bamio import records_from_aln, write_bam, write_phased_vcf, write_u_vcf

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "example")


def tagged(tmp_path, n_windows=4, coverage=30, seed=22, len_scale=0.5, contig="chrS"):
    """Pre-haplotagged BAM (HP tags, HP:i:0 and missing de now and then)."""
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    aln = make_aln_batch(AlnSpec(n_windows=n_windows, coverage=coverage, seed=seed, len_scale=len_scale),
                         workers=min(4, n_windows))
    recs = records_from_aln(aln, hp_zero_every=11, de_absent_every=13)
    bam = str(tmp_path / "t.bam")
    write_bam(bam, [(contig, 200_000_000)], recs)
    vcf = str(tmp_path / "t.vcf")
    write_phased_vcf(vcf, contig, list(zip(aln.win_start.tolist(), aln.win_end.tolist())))
    return aln, recs, bam, vcf


def untagged(tmp_path, n_windows=3, coverage=60, seed=71, len_scale=1.0, contig="chrS"):
    """-u fixture: het SNVs with MD tags, no HP tags in the BAM."""
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    aln = make_aln_batch(AlnSpec(n_windows=n_windows, coverage=coverage, seed=seed, het_snv_rate=0.001,
                                 untag_frac=0.0, len_scale=len_scale), workers=min(4, n_windows))
    aln.hp[:] = 254
    recs = records_from_aln(aln)
    bam = str(tmp_path / "u.bam")
    write_bam(bam, [(contig, 400_000_000)], recs)
    vcf = str(tmp_path / "u.vcf")
    write_u_vcf(vcf, contig, aln)
    return aln, recs, bam, vcf


def example(tmp_path, coverage=60, seed=6):
    """The reference's example VCF with a synthetic chr6 BAM over its gap,
    planted TRANS (the golden run's decision)."""
    import oracle
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    vcf = os.path.join(GOLD, "variants.vcf.gz")
    gaps = oracle.vcf_gaps(vcf)
    (s, e), = gaps[0]["gaps"]
    aln = make_aln_batch(AlnSpec(n_windows=1, coverage=coverage, seed=seed, windows_at=((s, e),), orient_at=(1,)),
                         workers=1)
    recs = records_from_aln(aln)
    bam = str(tmp_path / "phased.bam")
    write_bam(bam, [("chr6", 170_805_979)], recs)
    return aln, recs, bam, vcf, gaps
