"""f1 on the device: pf_batch_upload_bam (BGZF inflate, record chain, record
decode, window chunk walk and gather on the GPU) against the host reader
pf_bam_fetch_windows on the same BAM -- the batch's record arrays, qnames and
raw HP values bit for bit, then the methphase decisions.  BAMs are written by
the test-side writer (tests/_bamio.py, htslib's block and index rules)."""
import struct

import numpy as np
import pytest

from tests import _bamio
from tests._fixtures import tagged

pytestmark = pytest.mark.gpu


def _compare(host, hqn, hinfo, db, dqn, dinfo):
    assert np.array_equal(dinfo["win_rec_off"], host.win_rec_off)
    d = db.debug_recs()
    for k in ("flag", "mapq", "pos", "l_qseq", "hp", "cigar_off", "mm_off", "ml_off"):
        assert np.array_equal(d[k], getattr(host, k)), k
    for k in ("cigar", "mm", "ml"):                    # the arrays' used parts (an empty batch keeps a pad element)
        n = int(getattr(host, k + "_off")[-1])
        assert np.array_equal(d[k], getattr(host, k)[:n]), k
    assert np.array_equal(d["de"].view(np.uint32), host.de.view(np.uint32))
    so = d["seq_off"]
    for i in range(host.n_recs):
        nb = (int(host.l_qseq[i]) + 1) // 2
        a = host.seq[host.seq_off[i]:host.seq_off[i] + nb].copy()
        if host.l_qseq[i] & 1:
            a[-1] &= 0xF0                              # the slice's pad nibble is 0 (pf_load.h)
        b = d["seq"][so[i]:so[i] + nb]
        assert np.array_equal(a, b), i
        assert not d["seq"][so[i] + nb:so[i + 1]].any()
    assert dqn == hqn
    assert np.array_equal(dinfo["hp_tag"], hinfo["hp_tag"])
    assert dinfo["n_truncated"] == hinfo["n_truncated"]


def _both(ctx, bam, chrom, ws, we, cfg, lcfg, **kw):
    from pomfret_amd.bam import BamFile
    with BamFile(bam) as b:
        host, hqn, hinfo = b.fetch_windows(chrom, ws, we, threads=4)
        db, dqn, dinfo = b.fetch_windows_device(ctx, cfg, chrom, ws, we, lcfg, **kw)
    return host, hqn, hinfo, db, dqn, dinfo


@pytest.mark.parametrize("ring", [None, ("196608", "77777"), ("98304", "98304")])
def test_device_fetch_tagged(gpu_ctx, tmp_path, monkeypatch, ring):
    """(ring: the staging ring's segment and read-piece sizes forced small;
    the fetch's many runs make the pieces run-relative, so segments end where
    the next piece would overflow a slot.)"""
    from pomfret_amd import Config, LoadConfig
    if ring:
        monkeypatch.setenv("PF_INGEST_SEG", ring[0])
        monkeypatch.setenv("PF_INGEST_PIECE", ring[1])
    aln, recs, bam, vcf = tagged(tmp_path, n_windows=4, coverage=30)
    cfg, lcfg = Config.from_coverage(30, given=False), LoadConfig()
    # the gap windows, plus windows shifted into their neighbours' readback
    ws = np.concatenate([aln.win_start, aln.win_start + 40_000, [0, 190_000_000]]).astype(np.uint32)
    we = np.concatenate([aln.win_end, aln.win_end + 40_000, [10, 190_000_010]]).astype(np.uint32)
    host, hqn, hinfo, db, dqn, dinfo = _both(gpu_ctx, bam, "chrS", ws, we, cfg, lcfg)
    assert host.n_recs > 0 and dinfo["n_blocks"] > 0
    _compare(host, hqn, hinfo, db, dqn, dinfo)
    out = db.run()
    ref = gpu_ctx.upload_aln(cfg, host, lcfg).run()
    for f in ("decision", "dir_table", "win_n_reads", "read_hp"):
        assert np.array_equal(getattr(out, f), getattr(ref, f)), f
    print(f"\n[fetch] {host.n_recs} records, {dinfo['n_blocks']} blocks, {dinfo['comp_bytes'] / 1e6:.1f} MB -> "
          f"{dinfo['inflated_bytes'] / 1e6:.1f} MB; inflate {dinfo['ms_inflate']:.3f} ms, chain "
          f"{dinfo['ms_chain']:.3f}, decode {dinfo['ms_decode']:.3f}, select+small {dinfo['ms_select']:.3f}, "
          f"build {dinfo['ms_build']:.3f}, total {dinfo['ms_total']:.1f} ms")


def _odd_records(tmp_path):
    """Records exercising the decoder: Mm/Ml tags, an ML of another type, a
    malformed tag ending the aux walk, a CG:B:I long CIGAR, a record of
    ~600 KB (spans many blocks: the plan must widen), a CIGAR/SEQ length
    mismatch (the fetch of its window ends there), HP:i:0 / missing de."""
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    aln = make_aln_batch(AlnSpec(n_windows=3, coverage=20, seed=9, len_scale=0.3), workers=1)
    recs = _bamio.records_from_aln(aln, hp_zero_every=7, de_absent_every=5)
    w1 = int(aln.win_rec_off[1])
    rng = np.random.default_rng(2)

    def ren(r, a, b):
        r.aux = r.aux.replace(a, b, 1)

    ren(recs[3], b"MMZ", b"MmZ")
    ren(recs[3], b"MLBC", b"MlBC")
    i = recs[5].aux.find(b"MLBC")                               # ML:B:S -- not B:C, the read gets no calls
    assert i >= 0
    cnt = struct.unpack_from("<I", recs[5].aux, i + 4)[0]
    recs[5].aux = recs[5].aux[:i] + b"MLBS" + struct.pack("<I", cnt) + bytes(2 * cnt) + recs[5].aux[i + 8 + cnt:]
    recs[7].aux = b"XXq\x01" + recs[7].aux                     # unknown type: the walk stops
    r = recs[9]                                                 # CG:B:I long CIGAR
    real = list(r.cigar)
    rl = _bamio.ref_len(real)
    r.cigar = [(r.l_seq << 4) | 4, (rl << 4) | 3]
    r.aux = r.aux + _bamio.aux_BI("CG", real)
    big = recs[11]                                              # ~600 KB record
    n = 400_000
    s = rng.integers(1, 16, n, dtype=np.uint8)
    big.l_seq = n
    big.seq = bytes((s[0::2] << 4) | s[1::2])
    big.cigar = [(n << 4) | 0]
    big.aux = _bamio.aux_i("HP", 1)
    bad = recs[w1 + 4]                                          # query length != l_seq
    bad.cigar = list(bad.cigar) + [(3 << 4) | 1]
    bam = str(tmp_path / "odd.bam")
    _bamio.write_bam(bam, [("chrS", 200_000_000)], recs)
    return aln, bam


@pytest.mark.parametrize("seg", [None, "98304", "4096"])
def test_device_fetch_odd_records(gpu_ctx, tmp_path, monkeypatch, seg):
    """(seg: the staging ring's segment size forced small -- every slot
    reused many times, blocks straddling segments scanned from the copied
    tail of the previous one, the ~600 KB record over many segments.)"""
    from pomfret_amd import Config, LoadConfig
    if seg:
        monkeypatch.setenv("PF_INGEST_SEG", seg)
    aln, bam = _odd_records(tmp_path)
    cfg, lcfg = Config.from_coverage(20, given=False), LoadConfig()
    host, hqn, hinfo, db, dqn, dinfo = _both(gpu_ctx, bam, "chrS", aln.win_start, aln.win_end, cfg, lcfg)
    assert hinfo["n_truncated"] >= 1
    _compare(host, hqn, hinfo, db, dqn, dinfo)
    out = db.run()
    ref = gpu_ctx.upload_aln(cfg, host, lcfg).run()
    assert np.array_equal(out.decision, ref.decision)
    assert np.array_equal(out.read_hp, ref.read_hp)


def test_device_fetch_record_limit(gpu_ctx, tmp_path):
    from pomfret_amd import Config, LoadConfig
    from pomfret_amd.bam import BamFile
    aln, recs, bam, vcf = tagged(tmp_path, n_windows=3, coverage=30, seed=4)
    cfg = Config.from_coverage(30, given=False)
    with BamFile(bam) as b:
        host, _, _ = b.fetch_windows("chrS", aln.win_start, aln.win_end)
        per = np.diff(host.win_rec_off.astype(np.int64))
        lim = int(np.sort(per)[1])                           # the largest window is over the limit
        db, qn, info = b.fetch_windows_device(gpu_ctx, cfg, "chrS", aln.win_start, aln.win_end, max_win_recs=lim)
    got = np.diff(info["win_rec_off"].astype(np.int64))
    assert np.array_equal(info["win_n_fetched"], per)
    assert np.array_equal(got, np.where(per > lim, 0, per))


@pytest.mark.parametrize("mode", ["tagged", "untagged", "report"])
def test_pipeline_device_vs_host_fetch(gpu_ctx, tmp_path, mode):
    """The C driver with the device fetch (default) and with --host-fetch:
    identical decisions, first-wins tag tables and output bytes."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import methphase_files, report_files
    from tests._fixtures import untagged
    if mode == "untagged":
        aln, recs, bam, vcf = untagged(tmp_path, n_windows=3, coverage=60)
        cfg = Config.from_coverage(60, given=False)
    else:
        aln, recs, bam, vcf = tagged(tmp_path, n_windows=4, coverage=30, seed=31)
        cfg = Config.from_coverage(30, given=False)
    outs = {}
    for hf in (False, True):
        pre = str(tmp_path / f"o{int(hf)}")
        if mode == "report":
            outs[hf] = (report_files(bam, vcf, pre, cov=30, chunk_size=20_000, chunk_stride=200_000,
                                     ctx=gpu_ctx, host_fetch=hf), pre)
        else:
            outs[hf] = (methphase_files(bam, vcf, pre, cfg, ctx=gpu_ctx, untagged=mode == "untagged", tsv=True,
                                        host_fetch=hf), pre)
    (rd, pd), (rh, ph) = outs[False], outs[True]
    assert np.array_equal(rd["decision"], rh["decision"])
    exts = [".report.tsv"] if mode == "report" else [".mp.gtf", ".mp.vcf", ".mp.tsv"]
    if mode != "report":
        assert rd["qname_hp"] == rh["qname_hp"]
    for e in exts:
        assert open(pd + e, "rb").read() == open(ph + e, "rb").read(), e


@pytest.mark.parametrize("seg", [None, "98304"])
def test_haptag_bam_vs_host(gpu_ctx, tmp_path, monkeypatch, seg):
    """-u pre-pass through the device fetch (pf_haptag_bam) against the host
    reader + K4 (pf_bam_fetch_contig_reads + pf_haptag_reads): the same reads
    (qnames, BAM order, secondary/unmapped skipped) and tags."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_bam import _u_bam
    from pomfret_amd.bam import BamFile, vcf_known_vars
    from pomfret_amd.synth_u import USpec
    if seg:
        monkeypatch.setenv("PF_INGEST_SEG", seg)
    known, reads, order, bam, vcf = _u_bam(tmp_path, USpec(n_reads=600, ref_len=400_000))
    kv = vcf_known_vars(vcf, "chrU")
    with BamFile(bam) as b:
        got, qn, _ = b.fetch_contig_reads("chrU")
        hp_d, qn_d, info = b.haptag_device(gpu_ctx, "chrU", kv)
    assert qn_d == qn
    assert np.array_equal(hp_d, gpu_ctx.haptag_reads(kv, got))


@pytest.mark.parametrize("cov", [60])
def test_untagged_pipeline_device_prepass(gpu_ctx, tmp_path, cov):
    """The driver's -u run with the device pre-pass and device fetch equals the
    host-fetch run (decisions, the raw -u table, outputs)."""
    from pomfret_amd import Config
    from pomfret_amd.pipeline import methphase_files
    from tests._fixtures import untagged
    aln, recs, bam, vcf = untagged(tmp_path, n_windows=2, coverage=cov, seed=5)
    cfg = Config.from_coverage(cov, given=False)
    r = {hf: methphase_files(bam, vcf, str(tmp_path / f"u{int(hf)}"), cfg, ctx=gpu_ctx, untagged=True, host_fetch=hf)
         for hf in (False, True)}
    assert np.array_equal(r[False]["decision"], r[True]["decision"])
    assert r[False]["raw_hp"] == r[True]["raw_hp"]
    assert r[False]["qname_hp"] == r[True]["qname_hp"]


def test_device_fetch_contigs_and_eof(gpu_ctx, tmp_path):
    """Two contigs and unplaced reads at the end of the file: fetches that
    stop at a record of the next tid, windows reaching past the last record of
    a contig, the last contig's fetch running into the unplaced tail (tid -1)
    and into EOF, and an empty contig -- device fetch against the host reader."""
    from pomfret_amd import Config, LoadConfig
    from pomfret_amd.bam import BamFile
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    a1 = make_aln_batch(AlnSpec(n_windows=2, coverage=20, seed=41, len_scale=0.3), workers=1)
    a2 = make_aln_batch(AlnSpec(n_windows=2, coverage=20, seed=42, len_scale=0.3), workers=1)
    r1 = _bamio.records_from_aln(a1, tid=0, prefix="a")
    r2 = _bamio.records_from_aln(a2, tid=2, prefix="b")
    un = _bamio.records_from_aln(a2, tid=-1, prefix="u")[:25]
    for r in un:                                         # unplaced: no position, unmapped
        r.pos, r.flag, r.cigar = -1, 4, []
    bam = str(tmp_path / "multi.bam")
    _bamio.write_bam(bam, [("c1", 200_000_000), ("c_empty", 1_000_000), ("c3", 200_000_000)], r1 + r2 + un)
    cfg, lcfg = Config.from_coverage(20, given=False), LoadConfig()
    ends1 = int(max(r.pos for r in r1)) + 200_000
    cases = [("c1", np.concatenate([a1.win_start, [ends1, 0]]), np.concatenate([a1.win_end, [ends1 + 10, 5_000_000]])),
             ("c3", np.concatenate([a2.win_start, [int(max(r.pos for r in r2)) + 30_000]]),
              np.concatenate([a2.win_end, [199_000_000]])),
             ("c_empty", np.array([1000], np.uint32), np.array([2000], np.uint32))]
    for chrom, ws, we in cases:
        ws = np.asarray(ws, np.uint32)
        we = np.asarray(we, np.uint32)
        with BamFile(bam) as b:
            host, hqn, hinfo = b.fetch_windows(chrom, ws, we, threads=2)
            db, dqn, dinfo = b.fetch_windows_device(gpu_ctx, cfg, chrom, ws, we, lcfg)
        _compare(host, hqn, hinfo, db, dqn, dinfo)
        if host.n_recs:
            assert np.array_equal(db.run().decision, gpu_ctx.upload_aln(cfg, host, lcfg).run().decision)
        db.free()


def _cov_records(rng, lens, n_per, trunc_at=None):
    from tests._bamio import Rec, aux_f
    recs = []
    for tid, n in enumerate(n_per):
        for _ in range(n):
            L = int(rng.integers(5_000, 40_000))
            p = int(rng.integers(0, max(1, lens[tid] - 1000)))
            flag = int(rng.choice([0, 0, 0, 16, 256, 2048]))
            aux = aux_f("de", float(rng.choice([0.01, 0.05, 0.2]))) if rng.random() < 0.7 else b""
            recs.append(Rec(tid, p, f"t{tid}_{len(recs)}", flag=flag, mapq=int(rng.integers(0, 60)),
                            cigar=[(L << 4) | 0], seq=rng.integers(0, 256, (L + 1) // 2, np.uint8).tobytes(),
                            l_seq=L, aux=aux))
    recs.sort(key=lambda r: (r.tid, r.pos))
    if trunc_at is not None:                          # CIGAR and SEQ lengths differ: the pass stops there
        r = recs[trunc_at]
        r.flag = 0
        r.cigar = [((r.l_seq - 7) << 4) | 0]
    return recs


@pytest.mark.parametrize("piece", [0, 256 << 10])
def test_estimate_coverage_device(gpu_ctx, tmp_path, piece):
    """pf_bam_estimate_coverage_dev against the serial host pass: plain,
    an unplaced tail (the last contig keeps 0), an empty contig, a truncated
    record mid-file (later contigs 0), and pieces of 256 KiB compressed (a
    record counts in the piece its start falls in)."""
    from tests._bamio import Rec
    from pomfret_amd.bam import BamFile
    rng = np.random.default_rng(21)
    lens = [300_000, 1_000_000, 123_456, 60_000]
    refs = [("a", lens[0]), ("empty", lens[1]), ("b", lens[2]), ("c", lens[3])]
    base = _cov_records(rng, lens, [150, 0, 150, 60])
    un = [Rec(-1, -1, f"u{i}", flag=4, cigar=[], seq=bytes(50), l_seq=100) for i in range(3)]
    n_a = sum(r.tid == 0 for r in base)
    cases = {"plain": base, "unplaced": base + un,
             "trunc": _cov_records(np.random.default_rng(21), lens, [150, 0, 150, 60], trunc_at=n_a + 40) + un}
    for name, recs in cases.items():
        path = str(tmp_path / f"{name}.bam")
        _bamio.write_bam(path, refs, recs)
        with BamFile(path) as b:
            host = b.estimate_coverage()
            dev = b.estimate_coverage_device(gpu_ctx, piece)
            assert b.n_unplaced == (3 if name != "plain" else 0)
        assert dev == host, name
        assert host[0] > 0 and host[1] == 0
        assert (host[3] > 0) == (name == "plain")
