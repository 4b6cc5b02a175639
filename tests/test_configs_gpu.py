"""GPU parity on the BASELINE configurations and the parity traps that need
large or hand-made windows (VERDICT r01 "next round" 1 and 10):

  * configs[2]: a WGS-like 8,192-window record-level batch (30x, gap mix)
    through K0..K3 -- multi-GB arenas, u64 offsets, > 2^32 SEQ bytes --
    against the oracle on its distinct windows;
  * configs[3]: 60x `--bam-is-untagged` end to end from files
    (methphase_files(untagged=True): VCF known variants + BAM -> K4 pre-pass
    -> K0..K3 -> blocks, GTF/TSV/VCF), equal to the oracle pipeline in
    decisions, both qname tables and the output bytes;
  * configs[0]: the reference's example VCF at `-c 60` with a synthetic chr6
    BAM covering its gap (planted TRANS, as the golden run decided), equal
    to the oracle pipeline and to the golden output.mp.vcf / .mp.gtf up to
    the documented differences of the older build;
  * the pre-haplotagged pipeline with output bytes and the qname table;
  * T8 (u16 site counters wrapping at 4096) and T6 (mmr_min_i wrapping to
    UINT32_MAX) on hand-worked windows;
  * the CLI's --gtf / --tsv phase blocks and -U (VERDICT r04 "next round" 1).
"""
import os
import subprocess

import numpy as np
import pytest

from tests import _fixtures as fx
from tests._bamio import records_from_aln
from tests._oracle_pipeline import methphase_files_oracle, report_oracle

pytestmark = pytest.mark.gpu

GOLD = fx.GOLD
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tile_aln(a, k):
    """k back-to-back copies of a record-level batch (same windows repeated)."""
    from pomfret_amd.abi import AlnBatch
    n = a.n_recs

    def toff(off):
        off = np.asarray(off, np.int64)
        tot = int(off[-1])
        return np.concatenate([off[:-1] + i * tot for i in range(k)] + [[k * tot]]).astype(np.uint64), tot

    out = {}
    for name in ("cigar", "seq", "mm", "ml"):
        off, tot = toff(getattr(a, name + "_off"))
        out[name + "_off"] = off
        out[name] = np.tile(getattr(a, name)[:tot], k)
    wro = a.win_rec_off.astype(np.int64)
    return AlnBatch(win_start=np.tile(a.win_start, k), win_end=np.tile(a.win_end, k),
                    win_rec_off=np.concatenate([wro[:-1] + i * n for i in range(k)] + [[k * n]]).astype(np.uint32),
                    flag=np.tile(a.flag, k), mapq=np.tile(a.mapq, k), pos=np.tile(a.pos, k),
                    l_qseq=np.tile(a.l_qseq, k), de=np.tile(a.de, k), hp=np.tile(a.hp, k), **out)


def test_wgs_8192_windows(oracle_lib, gpu_ctx):
    """configs[2]: 8,192 windows (512 distinct WGS-like windows at 30x with
    the 5-500 kb gap mix, 16 copies) in one record-level batch.  Every copy
    must reproduce the oracle's decisions, 2x2 tables, site/read counts and
    read tags of the distinct windows bit for bit."""
    from pomfret_amd import Config, LoadConfig
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    cfg, lcfg = Config.from_coverage(30, given=False), LoadConfig()
    base = make_aln_batch(AlnSpec(n_windows=512, coverage=30, seed=3000, gap_mix=True), workers=16)
    wb, _ = oracle_lib.load_reads(lcfg, base)
    ref = oracle_lib.methphase(cfg, wb, n_threads=16)
    K = 16
    big = _tile_aln(base, K)
    assert big.n_windows == 8192 and int(big.seq_off[-1]) > 2 ** 32
    del base
    db = gpu_ctx.upload_aln(cfg, big, lcfg)
    del big
    out = db.run()
    W, R = wb.n_windows, wb.n_reads
    assert out.read_hp.shape[0] == K * R
    for f in ("decision", "win_n_sites", "win_n_reads"):
        got = getattr(out, f).reshape(K, W)
        for k in range(K):
            assert np.array_equal(got[k], getattr(ref, f)), f"copy {k}: {f}"
    tab = out.dir_table.reshape((K, W) + out.dir_table.shape[1:])
    for k in range(K):
        assert np.array_equal(tab[k], ref.dir_table), f"copy {k}: dir_table"
    hp = out.read_hp.reshape(K, R)
    for k in range(K):
        assert np.array_equal(hp[k], ref.read_hp), f"copy {k}: read_hp"
    assert (ref.decision >= 0).sum() > W // 2
    db.free()


def _compare_pipeline(res, ref, out_prefix):
    assert np.array_equal(res["decision"], ref["decision"])
    assert res["qname_hp"] == ref["qname_hp"]
    assert open(out_prefix + ".mp.gtf").read() == ref["gtf"]
    assert open(out_prefix + ".mp.tsv").read() == ref["tsv"]
    assert open(out_prefix + ".mp.vcf", "rb").read() == ref["vcf"]


def test_untagged_60x_end_to_end(oracle_lib, gpu_ctx, tmp_path):
    """configs[3] (`methphase -u` at 60x): het SNVs every ~1 kb outside the
    gaps with consistent CIGAR/MD/SEQ; the BAM carries no HP tags.  The K4
    pre-pass tags reads from the VCF, K0..K3 phase the gaps with those tags
    (blockjoin.c:1114-1122), and every output equals the oracle pipeline.
    One window per job: the next job's fetch overlaps the current kernels."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import methphase_files
    aln, recs, bam, vcf = fx.untagged(tmp_path)
    cfg = Config.from_coverage(60, given=True)
    out = str(tmp_path / "out")
    res = methphase_files(bam, vcf, out, cfg, ctx=gpu_ctx, untagged=True, tsv=True, job_windows=1)
    ref = methphase_files_oracle(bam, vcf, cfg, untagged=True, recs_by_contig={"chrS": recs})
    _compare_pipeline(res, ref, out)
    assert res["raw_hp"] == ref["raw_hp"]
    assert (ref["decision"] >= 0).sum() >= 2
    joined = ref["decision"] >= 0
    assert np.array_equal(ref["decision"][joined], aln.meta["orient"][joined])


def test_tagged_pipeline_bytes(oracle_lib, gpu_ctx, tmp_path):
    """The pre-haplotagged pipeline (configs[1] shape, HP tags in the BAM):
    decisions, the joined windows' first-wins qname table and the GTF/TSV/VCF
    bytes equal the oracle pipeline."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import methphase_files
    aln, recs, bam, vcf = fx.tagged(tmp_path)
    cfg = Config.from_coverage(30, given=False)
    out = str(tmp_path / "out")
    res = methphase_files(bam, vcf, out, cfg, ctx=gpu_ctx, tsv=True)
    ref = methphase_files_oracle(bam, vcf, cfg, recs_by_contig={"chrS": recs})
    _compare_pipeline(res, ref, out)
    assert len(ref["qname_hp"]) > 0


def test_example_plumbing_c60(oracle_lib, gpu_ctx, tmp_path):
    """configs[0]: `methphase -c 60 --vcf example/variants.vcf.gz` with a
    synthetic chr6 BAM over the example's gap (the reference's phased.bam is
    not in the repo).  Reads are planted TRANS, as the golden run joined;
    the outputs equal the oracle pipeline, and the golden output.mp.vcf /
    .mp.gtf up to the two documented differences of the older build."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import methphase_files
    aln, recs, bam, vcf, gaps = fx.example(tmp_path)
    cfg = Config.from_coverage(60, given=True)
    out = str(tmp_path / "out")
    res = methphase_files(bam, vcf, out, cfg, ctx=gpu_ctx, tsv=True)
    ref = methphase_files_oracle(bam, vcf, cfg, recs_by_contig={"chr6": recs})
    _compare_pipeline(res, ref, out)
    assert res["decision"].tolist() == [1]
    _golden_check(out, gaps)


def _golden_check(out, gaps):
    got = open(out + ".mp.vcf", "rb").read().split(b"\n")
    gold = open(os.path.join(GOLD, "output.mp.vcf"), "rb").read().split(b"\n")
    assert len(got) == len(gold)
    diff = [i for i in range(len(got)) if got[i] != gold[i]]
    assert len(diff) == 1 and int(got[diff[0]].split(b"\t")[1]) == gaps[0]["abs_end"]
    gtf = open(out + ".mp.gtf").read()
    assert gtf.replace("\t.\t+", ".\t+", 1) == open(os.path.join(GOLD, "output.mp.gtf")).read()


def _cli(*args, timeout=300, env=None):
    exe = os.path.join(ROOT, "pomfret_amd", "pomfret-amd")
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout,
                          env=dict(os.environ, **env) if env else None)


def test_cli_methphase_example(oracle_lib, tmp_path):
    """The command-line drop-in: `pomfret-amd methphase -o out -c 60 --vcf
    example/variants.vcf.gz phased.bam` (configs[0]) writes the oracle
    pipeline's bytes."""
    from pomfret_amd import Config
    aln, recs, bam, vcf, gaps = fx.example(tmp_path)
    out = str(tmp_path / "cli")
    r = _cli("methphase", "-o", out, "-c", "60", "--vcf", vcf, "--output-tsv", "-t", "4", bam)
    assert r.returncode == 0, r.stderr
    ref = methphase_files_oracle(bam, vcf, Config.from_coverage(60, given=True), recs_by_contig={"chr6": recs})
    assert open(out + ".mp.gtf").read() == ref["gtf"]
    assert open(out + ".mp.tsv").read() == ref["tsv"]
    assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]
    _golden_check(out, gaps)


@pytest.mark.parametrize("per_gpu", [None, "1", "3"])
def test_cli_untagged_no_c(oracle_lib, tmp_path, per_gpu):
    """`pomfret-amd methphase -u` without -c: the K4 pre-pass, then the
    per-contig parameters from the coverage estimate (4357-4374).  per_gpu:
    PF_DEV_CONTEXTS (default 2 contexts per GPU; the window jobs of one
    context read the -u arenas another context of the GPU kept)."""
    from pomfret_amd import Config
    from pomfret_amd.bam import BamFile
    aln, recs, bam, vcf = fx.untagged(tmp_path, n_windows=2, coverage=40)
    out = str(tmp_path / "cli")
    r = _cli("methphase", "-u", "-o", out, "--vcf", vcf, "--job-windows", "1", bam,
             env={"PF_DEV_CONTEXTS": per_gpu} if per_gpu else None)
    assert r.returncode == 0, r.stderr
    with BamFile(bam) as b:
        cfg = Config.from_coverage(b.estimate_coverage()[0], given=False)
    ref = methphase_files_oracle(bam, vcf, cfg, untagged=True, recs_by_contig={"chrS": recs})
    assert open(out + ".mp.gtf").read() == ref["gtf"]
    assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]


def test_report_gpu_matches_oracle(oracle_lib, gpu_ctx, tmp_path):
    """`pomfret report` (a14, main_methreport 4901-5089) on the device:
    chunk windows inside the phased blocks, report.tsv rows and totals equal
    the oracle's; the CLI writes the same file."""
    from pomfret_amd.pipeline import report_files
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=3)
    out = str(tmp_path / "rep")
    res = report_files(bam, vcf, out, cov=30, chunk_size=10_000, chunk_stride=50_000, ctx=gpu_ctx)
    text = open(out + ".report.tsv").read()
    assert text == report_oracle(bam, vcf, 30, 10_000, 50_000)
    assert sum(res["counts"].values()) == text.count("\n") > 0
    r = _cli("report", "-o", str(tmp_path / "rep2"), "-c", "30", "--chunk-size", "10000", "--chunk-stride", "50000",
             "--vcf", vcf, bam)
    assert r.returncode == 0, r.stderr
    assert open(str(tmp_path / "rep2") + ".report.tsv").read() == text
    assert f"Total N={text.count(chr(10))} regions" in r.stdout


def test_report_200x_record_level(oracle_lib, gpu_ctx, tmp_path):
    """BASELINE configs[4] at record level (VERDICT r02 "next round" 8):
    `pomfret report -c 200 --chunk-size 10000 --chunk-stride 5000` on a 200x
    pre-haplotagged pileup (tests/_genome.report_spec: 50 chunk windows of
    ~1,700 reads each, cov_for_selection 21, n_cand 51) from BAM files
    through the device fetch and K0..K3, against the oracle (main_methreport,
    blockjoin.c:4966-4993, 5044-5078): every report.tsv row and the totals."""
    from pomfret_amd.pipeline import report_files
    from tests import _genome
    g = _genome.write_genome(str(tmp_path / "r200"), _genome.report_spec(), workers=4)
    out = str(tmp_path / "rep")
    res = report_files(g["bam"], g["vcf"], out, cov=200, chunk_size=10_000, chunk_stride=5_000, ctx=gpu_ctx)
    text = open(out + ".report.tsv").read()
    ref = report_oracle(g["bam"], g["vcf"], 200, 10_000, 5_000)
    assert text == ref
    n = text.count("\n")
    assert n >= 20 and sum(res["counts"].values()) == n
    assert res["counts"]["correct"] >= n // 2 and res["counts"]["fail"] > 0     # undecided chunks are present


def test_oversized_window_left_undecided(oracle_lib, gpu_ctx, tmp_path):
    """A window with more records than the device's per-window limit (65,535)
    is left undecided with a warning; the other windows of the run are
    unaffected."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import methphase_files
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    from tests._bamio import Rec, write_bam, write_phased_vcf
    aln = make_aln_batch(AlnSpec(n_windows=2, coverage=30, seed=22, len_scale=0.5), workers=2)
    recs = records_from_aln(aln)
    s1 = int(aln.win_start[1])
    junk = [Rec(0, s1 + 1000 + (i % 20000), f"j{i}", cigar=[(20 << 4) | 0], seq=bytes([0x12] * 10), l_seq=20)
            for i in range(66_000)]
    allr = sorted(recs + junk, key=lambda r: r.pos)
    bam = str(tmp_path / "big.bam")
    write_bam(bam, [("chrS", 200_000_000)], allr)
    vcf = str(tmp_path / "big.vcf")
    write_phased_vcf(vcf, "chrS", list(zip(aln.win_start.tolist(), aln.win_end.tolist())))
    cfg = Config.from_coverage(30, given=False)
    res = methphase_files(bam, vcf, str(tmp_path / "o"), cfg, ctx=gpu_ctx)
    ref = methphase_files_oracle(bam, vcf, cfg, recs_by_contig={"chrS": allr})
    assert res["n_limit"] == 1 and res["decision"][1] == -1
    assert res["decision"][0] == ref["decision"][0]


def test_t8_counter_wrap_gpu(oracle_lib, gpu_ctx):
    """T8 on the device: K12's site counts wrap at 4096 like the reference's
    u16 counters; sites worked out by hand (tests/_cases.T8_SITES)."""
    from tests._cases import T8_CFG, T8_SITES, t8_counter_wrap
    b = t8_counter_wrap()
    db = gpu_ctx.upload(T8_CFG, b)
    for d in (0, 1):
        real, _, _ = db.debug_sites(0, d)
        assert real.tolist() == T8_SITES
    out = db.run()
    ref = oracle_lib.methphase(T8_CFG, b)
    for f in ("decision", "dir_table", "win_n_sites", "win_n_reads", "read_hp"):
        assert np.array_equal(getattr(out, f), getattr(ref, f)), f
    db.free()


def test_t6_range_wrap_gpu(oracle_lib, gpu_ctx):
    """T6 on the device: with every site right of e, direction 1 inserts no
    read (mmr_min_i wrapped to UINT32_MAX) while direction 0 does; the whole
    result equals the oracle."""
    from pomfret_amd import Config
    from tests._cases import t6_range_wrap
    cfg = Config(k=3, k_span=5000, cov_for_selection=4, cov_for_runtime=8, n_cand=8)
    b = t6_range_wrap()
    db = gpu_ctx.upload(cfg, b)
    out = db.run()
    st = db.stats()
    assert st[0, 1, 0] == 0 and st[0, 0, 0] > 0          # in-range methmer lookups per direction
    ref = oracle_lib.methphase(cfg, b)
    for f in ("decision", "dir_table", "dir_join", "win_n_sites", "read_hp"):
        assert np.array_equal(getattr(out, f), getattr(ref, f)), f
    assert out.dir_join[0, 1] == -1
    db.free()


def test_cli_write_bam_and_varhaptag(oracle_lib, tmp_path):
    """f4 on the device: `methphase -u --write-bam` writes {prefix}.mp.bam +
    .bai whose HP tags follow output_modify_bam over the oracle pipeline's
    tables (tests/test_bamw.py restates it), and `varhaptag -o out.bam vcf bam`
    writes the K4 tags of the oracle's -u pre-pass (main_varhaptag)."""
    from pomfret_amd import Config, _lib
    from tests.test_bamw import _restate_methphase, aux_update_int, hp_tag_raw, parse_bam, qname
    aln, recs, bam, vcf = fx.untagged(tmp_path, n_windows=2, coverage=30, len_scale=0.6)
    out = str(tmp_path / "wb")
    r = _cli("methphase", "-u", "-c", "30", "-o", out, "--vcf", vcf, "--write-bam", bam)
    assert r.returncode == 0, r.stderr
    ref = methphase_files_oracle(bam, vcf, Config.from_coverage(30, given=True), untagged=True,
                                 recs_by_contig={"chrS": recs})
    assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]
    g = _lib.Gaps(vcf)
    b = _lib.Blocks(g, ref["decision"])
    _, bodies_in, _, _ = parse_bam(bam)
    _, bodies_out, _, _ = parse_bam(out + ".mp.bam")
    hp = _restate_methphase(bodies_in, [0] * len(bodies_in), g.contigs(), b.contigs(), ref["qname_hp"],
                            ref["raw_hp"], tid_names=("chrS",))
    assert len(bodies_out) == len(bodies_in)
    for bi, bo, h in zip(bodies_in, bodies_out, hp):
        assert bo == aux_update_int(bi, h + 1)
    assert os.path.getsize(out + ".mp.bam.bai") > 0
    vb = str(tmp_path / "vh.bam")
    r = _cli("varhaptag", "-o", vb, vcf, bam)
    assert r.returncode == 0, r.stderr
    lines = open(vb + ".varhaptag.tsv").read().split("\n")[1:-1]
    _, bodies_v, _, _ = parse_bam(vb)
    for bi, bo, line in zip(bodies_in, bodies_v, lines):
        h = ref["raw_hp"].get(qname(bi), 254)
        assert line == f"{qname(bi)}\t{hp_tag_raw(bi) + 1}\t{h + 1}"
        assert bo == aux_update_int(bi, h + 1)


def _cli_blocks(aln, merge_pair):
    from tests.test_pipeline import _shifted
    return _shifted(aln, merge_pair=merge_pair)


@pytest.mark.parametrize("fmt", ["gtf", "tsv"])
def test_cli_gtf_tsv_blocks(oracle_lib, tmp_path, fmt):
    """`pomfret-amd methphase --gtf blocks.gtf --vcf v.vcf` and `--tsv
    blocks.tsv` (no --vcf: no VCF written, 4706): windows from the block file
    (main_blockjoin 4661-4666), GTF / TSV / VCF bytes equal the oracle
    pipeline's.  The no-VCF run also takes --write-bam, which the reference
    honours with or without a VCF (4714-4731): its records carry the HP tags
    output_modify_bam gives over the oracle's tables."""
    from pomfret_amd import Config, _lib
    from pomfret_amd.pipeline import INTERVALS_GTF, INTERVALS_TSV
    from tests.test_bamw import _restate_methphase, aux_update_int, parse_bam
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=4)
    cfg = Config.from_coverage(30, given=True)
    for with_vcf in (True, False):
        gtf, tsvp = fx.blocks_files(tmp_path, {"chrS": _cli_blocks(aln, not with_vcf)}, name=f"b{with_vcf}")
        iv = (gtf, INTERVALS_GTF) if fmt == "gtf" else (tsvp, INTERVALS_TSV)
        out = str(tmp_path / f"cli{int(with_vcf)}")
        args = ["methphase", "-o", out, "-c", "30", f"--{fmt}", iv[0], "--output-tsv"]
        if with_vcf:
            args += ["--vcf", vcf]
        else:
            args += ["--write-bam"]
        r = _cli(*args, bam)
        assert r.returncode == 0, r.stderr
        ref = methphase_files_oracle(bam, vcf if with_vcf else None, cfg, recs_by_contig={"chrS": recs},
                                     intervals=iv)
        assert (ref["decision"] >= 0).sum() >= 2
        assert open(out + ".mp.gtf").read() == ref["gtf"]
        assert open(out + ".mp.tsv").read() == ref["tsv"]
        if with_vcf:
            assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]
            assert "multiple phase block files" in r.stderr
        else:
            assert not os.path.exists(out + ".mp.vcf")
            g = _lib.Gaps(iv[0], fmt=iv[1])
            b = _lib.Blocks(g, ref["decision"])
            _, bodies_in, _, _ = parse_bam(bam)
            _, bodies_out, _, _ = parse_bam(out + ".mp.bam")
            hp = _restate_methphase(bodies_in, [0] * len(bodies_in), g.contigs(), b.contigs(), ref["qname_hp"],
                                    None, tid_names=("chrS",))
            assert len(bodies_out) == len(bodies_in)
            assert all(bo == aux_update_int(bi, h + 1) for bi, bo, h in zip(bodies_in, bodies_out, hp))
            assert os.path.getsize(out + ".mp.bam.bai") > 0


def test_cli_untagged_gtf_input_tagging(oracle_lib, tmp_path):
    """`pomfret-amd methphase -u -U --gtf blocks.gtf --vcf v.vcf`: K4 tags the
    reads from the VCF's variants, the GTF's blocks (with a dropped interval
    whose variants the rescue phases) define the windows, and -U writes
    {prefix}.mp.input_haptag.tsv; every file equals the oracle pipeline's."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import INTERVALS_GTF
    aln, recs, bam, vcf = fx.untagged(tmp_path, n_windows=2, coverage=30, len_scale=0.6)
    gtf, _ = fx.blocks_files(tmp_path, {"chrS": _cli_blocks(aln, True)})
    out = str(tmp_path / "u")
    r = _cli("methphase", "-u", "-U", "-c", "30", "-o", out, "--gtf", gtf, "--vcf", vcf, "--output-tsv", bam)
    assert r.returncode == 0, r.stderr
    ref = methphase_files_oracle(bam, vcf, Config.from_coverage(30, given=True), untagged=True,
                                 recs_by_contig={"chrS": recs}, intervals=(gtf, INTERVALS_GTF))
    assert open(out + ".mp.gtf").read() == ref["gtf"]
    assert open(out + ".mp.tsv").read() == ref["tsv"]
    assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]
    assert open(out + ".mp.input_haptag.tsv").read() == ref["input_haptag"]
    # -U without -u writes nothing (4494), and an empty block file terminates (4474-4477)
    r = _cli("methphase", "-U", "-c", "30", "-o", str(tmp_path / "t"), "--vcf", vcf, bam)
    assert r.returncode == 0 and not os.path.exists(str(tmp_path / "t") + ".mp.input_haptag.tsv")
    empty = str(tmp_path / "empty.gtf")
    open(empty, "w").write("# nothing\n")
    r = _cli("methphase", "-c", "30", "-o", str(tmp_path / "e"), "--gtf", empty, bam)
    assert r.returncode == 1 and "No intervals loaded" in r.stderr
