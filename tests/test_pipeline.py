"""The C pipeline driver on the CPU (no device): plan, job results, merge
and writers of pf_pipeline.c, with every job's compute supplied by the
oracle (tests/_oracle_pipeline.oracle_job_runner) -- the same results a
device run exports.  Checked against the oracle pipeline end to end:
decisions, the first-wins qname tables, GTF/TSV/VCF bytes, report.tsv.
The device path of the same driver is tests/test_configs_gpu.py."""
import os
import subprocess

import numpy as np
import pytest

from tests import _fixtures as fx
from tests._oracle_pipeline import methphase_files_oracle, oracle_job_runner, report_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_plan(plan, runner):
    from pomfret_amd.pipeline import JOB_HAPTAG, JOB_WINDOWS
    if plan.opts.untagged:
        for j in range(plan.n_jobs(JOB_HAPTAG)):
            plan.set_result(JOB_HAPTAG, j, runner(plan, JOB_HAPTAG, j))
        plan.merge_raw()
    for j in range(plan.n_jobs(JOB_WINDOWS)):
        plan.set_result(JOB_WINDOWS, j, runner(plan, JOB_WINDOWS, j))
    plan.finish()


def _compare(out_prefix, plan, ref):
    assert np.array_equal(plan.decisions(), ref["decision"])
    assert plan.qname_hp() == ref["qname_hp"]
    assert open(out_prefix + ".mp.gtf").read() == ref["gtf"]
    assert open(out_prefix + ".mp.tsv").read() == ref["tsv"]
    assert open(out_prefix + ".mp.vcf", "rb").read() == ref["vcf"]


def test_tags_first_wins():
    from pomfret_amd.pipeline import Tags
    t = Tags()
    assert t.put_first(["a", "b", "a", "c"], [0, 1, 1, 254]) == 3
    assert t.put_first(["b", "d"], [0, 0]) == 1
    assert t.to_dict() == {"a": 0, "b": 1, "c": 254, "d": 0}
    assert t.get(["d", "zz", "a"], 254).tolist() == [0, 254, 0]
    many = [f"read{i}" for i in range(20000)]
    assert t.put_first(many, np.arange(20000) % 2) == 20000 and len(t) == 20004
    assert t.get(many[::997], 7).tolist() == [i % 2 for i in range(0, 20000, 997)]
    t.close()


@pytest.mark.parametrize("job_windows", [1, 3, 0])
def test_plan_tagged_matches_oracle(oracle_lib, tmp_path, job_windows):
    from pomfret_amd import Config
    from pomfret_amd.pipeline import JOB_WINDOWS, Plan, make_opts
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=4)
    cfg = Config.from_coverage(30, given=False)
    out = str(tmp_path / "o")
    plan = Plan(make_opts(bam, vcf, out, cfg, tsv=True, job_windows=job_windows))
    n = plan.n_jobs(JOB_WINDOWS)
    assert n == (4 if job_windows == 1 else 2 if job_windows == 3 else 1)
    _run_plan(plan, oracle_job_runner(bam, vcf))
    _compare(out, plan, methphase_files_oracle(bam, vcf, cfg, recs_by_contig={"chrS": recs}))
    plan.close()


def test_plan_untagged_matches_oracle(oracle_lib, tmp_path):
    from pomfret_amd import Config
    from pomfret_amd.pipeline import JOB_HAPTAG, Plan, make_opts
    aln, recs, bam, vcf = fx.untagged(tmp_path, n_windows=2, coverage=30, len_scale=0.6)
    cfg = Config.from_coverage(30, given=True)
    out = str(tmp_path / "o")
    plan = Plan(make_opts(bam, vcf, out, cfg, untagged=True, tsv=True, job_windows=1))
    assert plan.n_jobs(JOB_HAPTAG) == 1
    _run_plan(plan, oracle_job_runner(bam, vcf))
    ref = methphase_files_oracle(bam, vcf, cfg, untagged=True, recs_by_contig={"chrS": recs})
    _compare(out, plan, ref)
    assert plan.raw_hp() == ref["raw_hp"]
    plan.close()


def test_plan_example_estimated_coverage(oracle_lib, tmp_path):
    """No -c: per-contig parameters from the coverage estimate
    (blockjoin.c:4357-4374); the example VCF's contigs absent from the BAM."""
    from pomfret_amd import Config
    from pomfret_amd.bam import BamFile
    from pomfret_amd.pipeline import Plan, make_opts
    aln, recs, bam, vcf, gaps = fx.example(tmp_path)
    out = str(tmp_path / "o")
    plan = Plan(make_opts(bam, vcf, out, None, tsv=True))
    with BamFile(bam) as b:
        est = b.estimate_coverage()[b.tid("chr6")]
    cfg = Config.from_coverage(est, given=False)
    _run_plan(plan, oracle_job_runner(bam, vcf))
    assert plan.job_info(0, 0)["cfg"] == cfg
    _compare(out, plan, methphase_files_oracle(bam, vcf, cfg, recs_by_contig={"chr6": recs}))
    plan.close()


def test_report_plan_matches_oracle(oracle_lib, tmp_path, capfd):
    from pomfret_amd.pipeline import MODE_REPORT, Plan, make_opts
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=3, len_scale=0.5)
    out = str(tmp_path / "r")
    for cov in (30, 0):
        plan = Plan(make_opts(bam, vcf, out, None, mode=MODE_REPORT, cov=cov, chunk_size=10_000,
                              chunk_stride=100_000, job_windows=2))
        _run_plan(plan, oracle_job_runner(bam, vcf))
        text = open(out + ".report.tsv").read()
        assert text == report_oracle(bam, vcf, cov, 10_000, 100_000)
        n = text.count("\n")
        c = plan.report_counts()
        assert n > 0 and c["correct"] + c["switch"] + c["fail"] == n
        assert f"Total N={n} regions" in capfd.readouterr().out
        plan.close()


def test_cli_parses_and_fails_loudly_without_a_device(tmp_path):
    """The CLI mirrors cli.c's checks; with no GPU visible it fails instead
    of falling back to a CPU path."""
    exe = os.path.join(ROOT, "pomfret_amd", "pomfret-amd")
    if not os.path.exists(exe):
        pytest.skip("CLI not built")
    r = subprocess.run([exe, "methphase", "-o", str(tmp_path / "o"), "x.bam"], capture_output=True, text=True)
    assert r.returncode == 1 and "cannot all be absent" in r.stderr
    r = subprocess.run([exe, "frobnicate"], capture_output=True, text=True)
    assert r.returncode == 1 and "unknown subcommand" in r.stderr
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=1, len_scale=0.3)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([exe, "methphase", "-o", str(tmp_path / "o"), "--vcf", vcf, "-c", "30", bam],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 1 and "failed" in r.stderr
    assert not os.path.exists(str(tmp_path / "o") + ".mp.gtf")


def test_genome_port_matches_oracle(oracle_lib, tmp_path):
    """BASELINE configs[3]'s shape at small scale (tests/_genome: 4 contigs,
    windows sharing reads, merged gaps): the CPU port of the driver (the
    bench's e2e_u CPU side: the product's plan / merge / writers, the serial
    host coverage pass, oracle jobs on a thread pool) equals the oracle
    pipeline, dropped-interval rescue included."""
    from tests import _genome
    from tests._oracle_pipeline import methphase_files_port
    g = _genome.write_genome(str(tmp_path / "g"), _genome.small_spec(seed=9), workers=4, keep_recs=True)
    out = str(tmp_path / "p")
    res, ph = methphase_files_port(g["bam"], g["vcf"], out, None, untagged=True, threads=4, tsv=True)
    ref = methphase_files_oracle(g["bam"], g["vcf"], None, untagged=True, recs_by_contig=g["recs_by_contig"])
    assert np.array_equal(res["decision"], ref["decision"]) and (ref["decision"] >= 0).sum() >= 5
    assert res["raw_hp"] == ref["raw_hp"] and list(res["qname_hp"].items()) == list(ref["qname_hp"].items())
    assert open(out + ".mp.gtf").read() == ref["gtf"]
    assert open(out + ".mp.tsv").read() == ref["tsv"]
    assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]
    assert ref["counts"][1] > 0 and set(ph) >= {"plan_s", "haptag_s", "windows_s", "total_s"}


def _shifted(aln, merge_pair=True):
    """GTF gaps that are not the VCF's: each window trimmed, plus (merge_pair)
    a split of the first window into two raw gaps < READBACK apart, which
    merge_close_intervals fuses back into one window with a dropped interval"""
    g = [(int(s) + 1500, int(e) - 2500) for s, e in zip(aln.win_start, aln.win_end)]
    if merge_pair:
        s, e = g[0]
        m = (s + e) // 2
        g[0:1] = [(s, m - 200), (m + 200, e)]
    return g


@pytest.mark.parametrize("fmt", ["gtf", "tsv"])
def test_plan_gtf_tsv_matches_oracle(oracle_lib, tmp_path, fmt):
    """--gtf / --tsv phase blocks (main_blockjoin 4661-4666): windows from the
    file, the VCF (when given) rewritten with those blocks and its variants in
    the dropped interval rescued; without --vcf no VCF is written (4706)."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import INTERVALS_GTF, INTERVALS_TSV, Plan, make_opts
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=4)
    cfg = Config.from_coverage(30, given=False)
    for with_vcf in (True, False):
        # a dropped interval only without the VCF: this fixture's records carry
        # no MD, which the rescue asserts on (1594-1596)
        gtf, tsvp = fx.blocks_files(tmp_path, {"chrS": _shifted(aln, merge_pair=not with_vcf)}, name=f"b{with_vcf}")
        iv = (gtf, INTERVALS_GTF) if fmt == "gtf" else (tsvp, INTERVALS_TSV)
        out = str(tmp_path / f"o{int(with_vcf)}")
        plan = Plan(make_opts(bam, vcf if with_vcf else None, out, cfg, tsv=True, intervals=iv))
        _run_plan(plan, oracle_job_runner(bam, vcf))
        ref = methphase_files_oracle(bam, vcf if with_vcf else None, cfg, recs_by_contig={"chrS": recs},
                                     intervals=iv)
        assert len(ref["decision"]) == 4 and (ref["decision"] >= 0).sum() >= 2
        from pomfret_amd import _lib
        assert len(_lib.interval_gaps(*iv)[0]["dropped"]) == (0 if with_vcf else 1)
        assert np.array_equal(plan.decisions(), ref["decision"])
        assert plan.qname_hp() == ref["qname_hp"]
        assert open(out + ".mp.gtf").read() == ref["gtf"]
        assert open(out + ".mp.tsv").read() == ref["tsv"]
        if with_vcf:
            assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]
        else:
            assert not os.path.exists(out + ".mp.vcf")
        plan.close()


def test_plan_untagged_gtf_input_tagging(oracle_lib, tmp_path):
    """`-u --gtf blocks.gtf --vcf v.vcf -U`: the VCF's variants haplotag the
    reads, the GTF's blocks define the windows (4445-4465), -U writes
    {prefix}.mp.input_haptag.tsv (4494-4517)."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import INTERVALS_GTF, JOB_HAPTAG, Plan, make_opts
    aln, recs, bam, vcf = fx.untagged(tmp_path, n_windows=2, coverage=30, len_scale=0.6)
    gtf, _ = fx.blocks_files(tmp_path, {"chrS": _shifted(aln)})
    cfg = Config.from_coverage(30, given=True)
    out = str(tmp_path / "o")
    plan = Plan(make_opts(bam, vcf, out, cfg, untagged=True, tsv=True, intervals=(gtf, INTERVALS_GTF),
                          write_input_tagging=True))
    assert plan.n_jobs(JOB_HAPTAG) == 1
    _run_plan(plan, oracle_job_runner(bam, vcf))
    ref = methphase_files_oracle(bam, vcf, cfg, untagged=True, recs_by_contig={"chrS": recs},
                                 intervals=(gtf, INTERVALS_GTF))
    _compare(out, plan, ref)
    assert plan.raw_hp() == ref["raw_hp"] and len(ref["raw_hp"]) > 0
    text = open(out + ".mp.input_haptag.tsv").read()
    assert text == ref["input_haptag"]
    assert text.count("\n") == len(recs) + 1 and "\t255\t" in text      # no HP tags in the input


def test_plan_multicontig_gtf_lacks_a_vcf_contig(oracle_lib, tmp_path):
    """A GTF without one of the VCF's contigs and in another contig order: the
    -u pre-pass still runs over the VCF's contigs (first wins in VCF order),
    the windows follow the GTF, and the rescue's known tables attribute the
    missing contig's lines to the contig before it (2150-2163)."""
    from pomfret_amd.pipeline import INTERVALS_GTF, JOB_HAPTAG, Plan, make_opts
    from pomfret_amd import Config
    bam, vcf, recs_by, alns = fx.multi_contig(tmp_path, untagged=True, len_scale=0.3)
    ga = [(int(s), int(e)) for s, e in zip(alns["chrA"].win_start, alns["chrA"].win_end)]
    gc = [(int(s) + 1000, int(e) - 1000) for s, e in zip(alns["chrC"].win_start, alns["chrC"].win_end)]
    s, e = gc[1]
    gc[1:2] = [(s, (s + e) // 2 - 100), ((s + e) // 2 + 100, e)]       # a dropped interval in chrC
    gtf, _ = fx.blocks_files(tmp_path, {"chrC": gc, "chrA": ga})
    cfg = Config.from_coverage(40, given=True)
    out = str(tmp_path / "o")
    plan = Plan(make_opts(bam, vcf, out, cfg, untagged=True, tsv=True, intervals=(gtf, INTERVALS_GTF),
                          write_input_tagging=True))
    names = sorted(plan.job_info(JOB_HAPTAG, j)["contig_name"] for j in range(plan.n_jobs(JOB_HAPTAG)))
    assert names == ["chrA", "chrB", "chrC"]                  # the VCF's contigs, not the GTF's
    _run_plan(plan, oracle_job_runner(bam, vcf))
    ref = methphase_files_oracle(bam, vcf, cfg, untagged=True, recs_by_contig=recs_by,
                                 intervals=(gtf, INTERVALS_GTF))
    _compare(out, plan, ref)
    assert plan.raw_hp() == ref["raw_hp"]
    assert open(out + ".mp.input_haptag.tsv").read() == ref["input_haptag"]
    from pomfret_amd import _lib
    assert [c["name"] for c in _lib.interval_gaps(gtf, INTERVALS_GTF)] == ["chrC", "chrA"]
