"""f1 on the GPU: records fetched by the host BAM reader (pf_bam_fetch_windows)
through K0..K3 equal the oracle's record-level path on the same records, and
the end-to-end pipeline (VCF gaps -> BAM fetch -> GPU -> blocks/GTF/VCF)
reproduces the oracle's decisions.  The BAM and VCF are written by the
test-side writer (tests/_bamio.py)."""
import os

import numpy as np
import pytest

from tests._bamio import records_from_aln, write_bam, write_phased_vcf

pytestmark = pytest.mark.gpu


def _fixture(tmp_path, n_windows=4, seed=21):
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    aln = make_aln_batch(AlnSpec(n_windows=n_windows, coverage=30, seed=seed, len_scale=0.5), workers=1)
    recs = records_from_aln(aln, hp_zero_every=11, de_absent_every=13)
    bam = str(tmp_path / "s.bam")
    write_bam(bam, [("chrS", 200_000_000)], recs)
    return aln, bam


def test_fetched_batch_parity(oracle_lib, gpu_ctx, tmp_path):
    from pomfret_amd import Config, LoadConfig
    from pomfret_amd.bam import BamFile
    aln, bam = _fixture(tmp_path)
    with BamFile(bam) as b:
        got, qn, info = b.fetch_windows("chrS", aln.win_start, aln.win_end, threads=4)
    assert info["n_truncated"] == 0 and got.n_recs > 0
    cfg, lcfg = Config.from_coverage(30, given=False), LoadConfig()
    wb, rec_read = oracle_lib.load_reads(lcfg, got)
    db = gpu_ctx.upload_aln(cfg, got, lcfg)
    assert np.array_equal(db.read_recs(), np.flatnonzero(rec_read != 0xFFFFFFFF))
    off, gpos, gcat, _, _ = db.debug_calls()
    assert np.array_equal(off, wb.read_call_off)
    out = db.run()
    ref = oracle_lib.methphase(cfg, wb, n_threads=8)
    for f in ("decision", "dir_table", "dir_join", "dir_which_way", "win_n_sites", "win_n_reads", "read_hp"):
        assert np.array_equal(getattr(ref, f), getattr(out, f)), f
    ref2 = oracle_lib.methphase_aln(cfg, lcfg, got, n_threads=8)
    assert np.array_equal(ref2.decision, out.decision)
    db.free()


def test_pipeline_end_to_end(oracle_lib, gpu_ctx, tmp_path):
    from pomfret_amd import Config, LoadConfig
    from pomfret_amd.bam import BamFile
    from pomfret_amd.pipeline import methphase_files
    aln, bam = _fixture(tmp_path, seed=22)
    wins = list(zip(aln.win_start.tolist(), aln.win_end.tolist()))
    vcf = str(tmp_path / "p.vcf")
    write_phased_vcf(vcf, "chrS", wins)
    cfg = Config.from_coverage(30, given=False)
    res = methphase_files(bam, vcf, str(tmp_path / "out"), cfg, ctx=gpu_ctx, tsv=True)
    with BamFile(bam) as b:
        got, qn, _ = b.fetch_windows("chrS", aln.win_start, aln.win_end)
    ref = oracle_lib.methphase_aln(cfg, LoadConfig(), got, n_threads=8)
    assert np.array_equal(res["decision"], ref.decision)
    assert (res["decision"] >= 0).any()
    for ext in (".mp.gtf", ".mp.tsv", ".mp.vcf"):
        assert os.path.getsize(str(tmp_path / "out") + ext) > 0


def test_u_ingest_gpu(oracle_lib, gpu_ctx, tmp_path):
    """-u pre-pass from files: VCF known variants + BAM contig reads -> K4."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_bam import _u_bam
    from pomfret_amd.bam import BamFile, vcf_known_vars
    from pomfret_amd.synth_u import USpec
    known, reads, order, bam, vcf = _u_bam(tmp_path, USpec(n_reads=300, ref_len=300_000))
    kv = vcf_known_vars(vcf, "chrU")
    with BamFile(bam) as b:
        got, qn, _ = b.fetch_contig_reads("chrU")
    hp = gpu_ctx.haptag_reads(kv, got)
    assert np.array_equal(hp, oracle_lib.haptag_reads(kv, got))
