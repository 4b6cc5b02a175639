"""f1: the host BAM reader (pf_bam_*) -- index parse pinned by the reference's
example BAI, region fetch against the overlap rule on BAM files written by
tests/_bamio.py (an independent writer), and the record fields the loader
needs.  CPU only."""
import os

import numpy as np
import pytest

import oracle
from pomfret_amd import LoadConfig
from pomfret_amd.bam import BamFile
from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
from _bamio import (Rec, aux_BC, aux_BI, aux_f, aux_i, aux_Z, endpos, expected_fetch, records_from_aln,
                    write_bam)

HERE = os.path.dirname(os.path.abspath(__file__))
EXAMPLE_BAI = os.path.join(HERE, "golden", "example", "phased.bam.bai")


def test_example_bai_pinned():
    # the reference's own example index (example/phased.bam.bai): 195 targets,
    # reads on target 5 only, 315 mapped / 0 unmapped in its pseudo-bin
    with BamFile(None, EXAMPLE_BAI) as b:
        assert b.n_targets == 195
        assert b.index_stats(5) == (315, 0)
        with pytest.raises(Exception):
            b.index_stats(0)


def _aln_records(n_windows=3, seed=5):
    aln = make_aln_batch(AlnSpec(n_windows=n_windows, coverage=8, seed=seed, len_scale=0.3, filt_frac=0.1),
                         workers=1)
    return aln, records_from_aln(aln, hp_zero_every=7, de_absent_every=5)


def _check_fetch(bam_path, recs, refs, chrom, starts, ends, readback, threads=1):
    tid = [n for n, _ in refs].index(chrom)
    with BamFile(bam_path) as b:
        got, qn, info = b.fetch_windows(chrom, starts, ends, readback=readback, threads=threads)
    exp = [expected_fetch(recs, tid, s, e, readback) for s, e in zip(starts, ends)]
    wro = got.win_rec_off
    assert wro[-1] == got.n_recs == sum(len(x) for x in exp)
    for w, ids in enumerate(exp):
        assert [qn[i] for i in range(wro[w], wro[w + 1])] == [recs[j].qname for j in ids], f"window {w}"
    return got, qn, info, exp


def test_fetch_windows_matches_overlap_rule(tmp_path):
    aln, recs = _aln_records()
    refs = [("chrA", 50_000_000), ("chrB", 50_000_000)]
    # a second contig with the same records shifted, to exercise tid stops
    recs2 = [Rec(tid=1, pos=r.pos + 1000, qname="b" + r.qname, flag=r.flag, mapq=r.mapq, cigar=r.cigar,
                 seq=r.seq, l_seq=r.l_seq, aux=r.aux) for r in recs[:200]]
    allr = recs + recs2
    p = str(tmp_path / "x.bam")
    write_bam(p, refs, allr)
    starts = [int(s) for s in aln.win_start] + [10, 1_000]
    ends = [int(e) for e in aln.win_end] + [20, 2_000]
    for rb in (50_000, 0, 123):
        got, qn, info, exp = _check_fetch(p, allr, refs, "chrA", starts, ends, rb)
        assert info["n_truncated"] == 0
    # threads do not change the result
    g1, q1, _, _ = _check_fetch(p, allr, refs, "chrA", starts, ends, 50_000, threads=1)
    g4, q4, _, _ = _check_fetch(p, allr, refs, "chrA", starts, ends, 50_000, threads=4)
    assert q1 == q4
    for f in ("pos", "flag", "cigar", "seq", "mm", "ml", "de", "hp", "cigar_off", "seq_off"):
        assert np.array_equal(getattr(g1, f), getattr(g4, f)), f
    _check_fetch(p, allr, refs, "chrB", [int(aln.win_start[0])], [int(aln.win_end[0])], 50_000)


_FETCH_DIGEST = r"""
import hashlib, sys
from pomfret_amd._lib import lib
from pomfret_amd.bam import BamFile
p, chrom, s, e = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
h = hashlib.sha256()
with BamFile(p) as b:
    got, qn, info = b.fetch_windows(chrom, [s], [e], readback=50_000, threads=2)
for f in ("pos", "flag", "cigar", "seq", "mm", "ml", "de", "hp", "cigar_off", "seq_off"):
    h.update(getattr(got, f).tobytes())
h.update("\n".join(qn).encode())
print(lib().pf_host_inflater(), got.n_recs, h.hexdigest())
"""


def test_host_inflaters_agree(tmp_path):
    """The host BGZF reader decodes with libdeflate when the system has it and
    with zlib otherwise (or under PF_HOST_ZLIB): both fetch the same bytes."""
    import subprocess
    import sys
    aln, recs = _aln_records(n_windows=2, seed=4)
    p = str(tmp_path / "z.bam")
    write_bam(p, [("c1", 40_000_000)], recs)
    s, e = int(aln.win_start[0]), int(aln.win_end[-1])
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for name, extra in (("default", {}), ("zlib", {"PF_HOST_ZLIB": "1"})):
        env = {k: v for k, v in os.environ.items() if k != "PF_HOST_ZLIB"}
        env.update(extra)
        env["PYTHONPATH"] = repo + os.pathsep + env.get("PYTHONPATH", "")
        r = subprocess.run([sys.executable, "-c", _FETCH_DIGEST, p, "c1", str(s), str(e)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        out[name] = r.stdout.split()
    assert out["zlib"][0] == "0"
    have_ldf = any(os.path.exists(os.path.join(d, "libdeflate.so.0"))
                   for d in ("/usr/lib/x86_64-linux-gnu", "/usr/lib64", "/usr/lib"))
    assert out["default"][0] == ("1" if have_ldf else "0")
    assert int(out["default"][1]) > 0
    assert out["default"][1:] == out["zlib"][1:]


def test_fetched_fields_equal_the_written_records(tmp_path):
    aln, recs = _aln_records(n_windows=2, seed=9)
    refs = [("c1", 40_000_000)]
    p = str(tmp_path / "y.bam")
    write_bam(p, refs, recs)
    with BamFile(p) as b:
        assert b.targets == ["c1"] and b.lengths == [40_000_000]
        assert b.tid("c1") == 0 and b.tid("nope") == -1
        mapped, unmapped = b.index_stats(0)
        assert mapped + unmapped == len(recs)
        got, qn, info = b.fetch_windows("c1", aln.win_start, aln.win_end)
    idx = {r.qname: i for i, r in enumerate(recs)}
    for k in range(got.n_recs):
        i = int(qn[k][1:])
        assert idx[qn[k]] == i
        assert got.pos[k] == aln.pos[i] and got.flag[k] == aln.flag[i] and got.mapq[k] == aln.mapq[i]
        assert got.l_qseq[k] == aln.l_qseq[i]
        c = got.cigar[got.cigar_off[k]:got.cigar_off[k + 1]]
        assert np.array_equal(c, aln.cigar[aln.cigar_off[i]:aln.cigar_off[i + 1]])
        lq = int(aln.l_qseq[i])
        assert bytes(got.seq[got.seq_off[k]:got.seq_off[k + 1]]) == bytes(aln.seq[aln.seq_off[i]:aln.seq_off[i] + (lq + 1) // 2])
        assert bytes(got.mm[got.mm_off[k]:got.mm_off[k + 1]]) == bytes(aln.mm[aln.mm_off[i]:aln.mm_off[i + 1]])
        assert bytes(got.ml[got.ml_off[k]:got.ml_off[k + 1]]) == bytes(aln.ml[aln.ml_off[i]:aln.ml_off[i + 1]])
        # HP: 0/1 round trip; 254 whether HP is absent or HP:i:0 (get_hp_from_aln)
        assert got.hp[k] == aln.hp[i]
        de_w = aln.de[i] >= 0 and i % 5 != 0
        assert got.de[k] == (np.float32(aln.de[i]) if de_w else np.float32(-1))
        assert info["hp_tag"][k] == (int(aln.hp[i]) + 1 if aln.hp[i] != 254 else (0 if i % 7 == 0 else -2**31))


def test_fetch_feeds_the_loader(tmp_path):
    """fetch -> oracle loader gives the same reads and calls as the loader on
    the records selected by the overlap rule directly."""
    aln, recs = _aln_records(n_windows=2, seed=3)
    refs = [("c1", 40_000_000)]
    p = str(tmp_path / "z.bam")
    write_bam(p, refs, recs)
    with BamFile(p) as b:
        got, qn, _ = b.fetch_windows("c1", aln.win_start, aln.win_end)
    # de values that were dropped from the tags are -1 in both
    lc = LoadConfig()
    wb_got, rr_got = oracle.load_reads(lc, got)
    exp_ids = [expected_fetch(recs, 0, int(s), int(e), 50_000) for s, e in zip(aln.win_start, aln.win_end)]
    flat = [i for ids in exp_ids for i in ids]
    assert [int(q[1:]) for q in qn] == flat
    assert wb_got.n_reads > 0 and wb_got.n_calls > 0


def test_cg_tag_and_truncation(tmp_path):
    """kSmN placeholder + CG:B:I restores the CIGAR (bam_tag2cigar); a record
    whose CIGAR query length differs from l_qseq ends the window's fetch
    (bam_read1 returns -4, sam_itr_next < 0)."""
    seq = bytes([0x12] * 50)            # 100 bases
    real = [(60 << 4) | 0, (2 << 4) | 2, (40 << 4) | 0]          # 60M2D40M
    recs = [
        Rec(0, 1000, "a", cigar=[(100 << 4) | 0], seq=seq, l_seq=100),
        Rec(0, 1100, "cg", cigar=[(100 << 4) | 4, (102 << 4) | 3], seq=seq, l_seq=100,
            aux=aux_BI("CG", real) + aux_i("HP", 1)),
        Rec(0, 1200, "b", cigar=[(100 << 4) | 0], seq=seq, l_seq=100),
        Rec(0, 5000, "bad", cigar=[(90 << 4) | 0], seq=seq, l_seq=100),   # qlen 90 != 100
        Rec(0, 5100, "c", cigar=[(100 << 4) | 0], seq=seq, l_seq=100),
        Rec(0, 40000, "u", flag=4, cigar=[], seq=seq, l_seq=100),         # unmapped, placed
    ]
    refs = [("c", 100_000)]
    p = str(tmp_path / "c.bam")
    write_bam(p, refs, recs)
    with BamFile(p) as b:
        got, qn, info = b.fetch_windows("c", [1050, 4000, 39990], [1150, 6000, 40001], readback=0, threads=2)
    w = got.win_rec_off
    assert qn[w[0]:w[1]] == ["a", "cg", "b"][:w[1] - w[0]] and "cg" in qn[w[0]:w[1]]
    k = qn.index("cg")
    assert list(got.cigar[got.cigar_off[k]:got.cigar_off[k + 1]]) == real
    assert got.hp[k] == 0
    assert qn[w[1]:w[2]] == []                 # "bad" stops the window before "c"
    assert info["n_truncated"] == 1
    assert qn[w[2]:w[3]] == ["u"]              # unmapped: end = pos + 1 (its own bin and
    assert endpos(40000, [], 4) == 40001       # linear-index window: "bad" is not read)


def test_errors(tmp_path):
    with pytest.raises(FileNotFoundError):
        BamFile(str(tmp_path / "missing.bam"))
    p = str(tmp_path / "e.bam")
    write_bam(p, [("c", 1000)], [])
    with BamFile(p) as b:
        with pytest.raises(Exception):
            b.fetch_windows("nope", [1], [2])
        got, qn, _ = b.fetch_windows("c", [1, 5], [2, 9])
        assert got.n_recs == 0 and list(got.win_rec_off) == [0, 0, 0]
    bad = tmp_path / "bad.bam"
    bad.write_bytes(b"not a bam")
    with pytest.raises(Exception):
        BamFile(str(bad), p + ".bai")


# ---------------------------------------------------------------- -u ingest
def _py_known(lines, contig):
    """insert_variant_from_vcf_line (blockjoin.c:1432-1543) restated for the
    test: strtok tokens, GT 'a|b' with a, b in {0,1}, SNP/DEL/INS rules."""
    nt4 = {c: i for i, c in enumerate("ACGT")}
    nt4.update({c.lower(): i for c, i in list(nt4.items())})
    out = []
    for s in lines:
        if s.startswith("#"):
            continue
        tok = [t for t in s.split("\t") if t]
        if not tok or tok[0] != contig or len(tok) < 10:
            continue
        pos = (int("".join(ch for ch in tok[1] if ch.isdigit()) or 0) - 1) & 0xFFFFFFFF
        ref, alt = tok[3], tok[4]
        fmt = tok[8].split(":")
        if "GT" not in fmt:
            continue
        smp = tok[9].split(":")
        i = fmt.index("GT")
        if i >= len(smp) or len(smp[i]) != 3:
            continue
        gt = smp[i]
        if gt[1] != "|" or gt[0] not in "01" or gt[2] not in "01":
            continue
        if len(ref) == 1 and len(alt) == 1:
            op, ln, ch = 1, 1, alt
        elif len(ref) == len(alt):
            continue
        elif len(ref) > len(alt):
            op, ln, ch = 3, len(ref) - len(alt), ref[1:]
            pos += 1
        else:
            op, ln, ch = 2, len(alt) - len(ref), alt[1:]
        out.append((pos, ln, op, int(gt[0]), [nt4.get(c, 4) for c in ch[:ln]]))
    return out


def _kv_list(kv):
    return [(int(kv.pos[i]), int(kv.len[i]), int(kv.op[i]), int(kv.haptag[i]),
             kv.chars[kv.char_off[i]:kv.char_off[i + 1]].tolist()) for i in range(len(kv.pos))]


def test_vcf_known_vars_rules(tmp_path):
    from pomfret_amd.bam import vcf_known_vars
    body = [
        "c1\t100\t.\tA\tG\t50\tPASS\t.\tGT:PS\t0|1:100",          # SNP, haptag 0
        "c1\t200\t.\tACGT\tA\t50\tPASS\t.\tGT\t1|0",              # DEL 3 at POS
        "c1\t300\t.\tC\tCTTA\t50\tPASS\t.\tPS:GT\t7:0|1",         # INS 3, GT second
        "c1\t400\t.\tAC\tGT\t50\tPASS\t.\tGT\t0|1",               # MNP: skipped
        "c1\t500\t.\tA\tG\t50\tPASS\t.\tGT\t0/1",                 # unphased
        "c1\t600\t.\tA\tG\t50\tPASS\t.\tGT\t.|1",
        "c1\t700\t.\tA\tC,G\t50\tPASS\t.\tGT\t1|0",               # multi-allelic: 'INS' ",G"
        "c2\t800\t.\tA\tG\t50\tPASS\t.\tGT\t0|1",                 # other contig
        "c1\t\t900\t.\tT\tA\t50\tPASS\t.\tGT\t1|0",               # empty token collapses
        "c1\t950\t.\tA\tG\t50\tPASS\t.\tGT:PS\t0|1",              # sample without PS: fine for GT
        "c1\t990\t.\tA\tG\t50\tPASS\t.\tPS:GT\t12",               # sample shorter than GT index
    ]
    hdr = ["##fileformat=VCFv4.2", "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS"]
    p = tmp_path / "k.vcf"
    p.write_text("\n".join(hdr + body) + "\n" + "c1\t999\t.\tA\tG\t50\tPASS\t.\tGT\t0|1")  # no final newline
    got = _kv_list(vcf_known_vars(str(p), "c1"))
    assert got == _py_known(body, "c1")
    assert [g[:3] for g in got] == [(99, 1, 1), (200, 3, 3), (299, 3, 2), (699, 2, 2), (899, 1, 1), (949, 1, 1)]
    assert got[1][4] == [1, 2, 3] and got[2][4] == [3, 3, 0] and got[3][4] == [4, 2]
    assert _kv_list(vcf_known_vars(str(p), "c2")) == _py_known(body, "c2")
    # '#' lines never reach insert_variant_from_vcf_line on the paths that
    # collect variants (load_intervals_from_file skips them, 2023-2026)
    bad = tmp_path / "b.vcf"
    bad.write_text("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\n" + body[0] + "\n")
    assert _kv_list(vcf_known_vars(str(bad), "c1")) == _py_known(body[:1], "c1")
    with pytest.raises(FileNotFoundError):
        vcf_known_vars(str(tmp_path / "missing.vcf"), "c1")


def test_vcf_known_vars_multi_attribution(tmp_path):
    """recover_variant_phase_in_dropped_intervals' tables over a GTF's contigs
    (var_storage branch of load_intervals_from_file, blockjoin.c:2150-2163):
    lines of a VCF contig the GTF lacks go to the last contig found (none
    before the first hit); with every VCF contig named, each table is the
    single-contig one."""
    from pomfret_amd.bam import vcf_known_vars, vcf_known_vars_multi
    from tests._oracle_pipeline import known_positions_multi
    body = ["x0\t50\t.\tA\tG\t50\tPASS\t.\tGT\t0|1",     # before any hit: dropped
            "c1\t100\t.\tA\tG\t50\tPASS\t.\tGT\t0|1",
            "c1\t200\t.\tACGT\tA\t50\tPASS\t.\tGT\t1|0",
            "c2\t30\t.\tA\tG\t50\tPASS\t.\tGT\t1|0",      # not in the GTF: appended to c1
            "c2\t40\t.\tA\tG\t50\tPASS\t.\tGT\t0/1",      #   (unphased: rejected there too)
            "c3\t70\t.\tC\tCTT\t50\tPASS\t.\tGT\t0|1",
            "c2\t90\t.\tA\tT\t50\tPASS\t.\tGT\t0|1"]      # follows c3: appended to c3
    p = tmp_path / "m.vcf"
    p.write_text("##x\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS\n" + "\n".join(body) + "\n")
    got = vcf_known_vars_multi(str(p), ["c3", "c1"])
    ref = known_positions_multi(str(p), ["c3", "c1"])
    assert [g.pos.tolist() for g in got] == [ref["c3"], ref["c1"]] == [[69, 89], [99, 200, 29]]
    allc = vcf_known_vars_multi(str(p), ["x0", "c1", "c2", "c3"])
    for name, kv in zip(["x0", "c1", "c2", "c3"], allc):
        assert _kv_list(kv) == _kv_list(vcf_known_vars(str(p), name))


def test_vcf_known_vars_example_fixture():
    """the reference's example/variants.vcf.gz (bgzipped): the C loader and
    the restatement agree on every contig it names"""
    import gzip
    from pomfret_amd.bam import vcf_known_vars
    path = os.path.join(HERE, "golden", "example", "variants.vcf.gz")
    lines = gzip.decompress(open(path, "rb").read()).decode().split("\n")[:-1]
    contigs = sorted({l.split("\t")[0] for l in lines if l and not l.startswith("#")})
    assert contigs
    n = 0
    for c in contigs:
        got = _kv_list(vcf_known_vars(path, c))
        assert got == _py_known(lines, c), c
        n += len(got)
    assert n > 0


def _u_bam(tmp_path, spec):
    from pomfret_amd.synth_u import make_u_batch
    from _bamio import write_phased_vcf  # noqa: F401
    known, reads, hap, vrecs = make_u_batch(spec, with_vcf=True)
    recs = []
    for i in range(len(reads.start)):
        cig = [int(x) for x in reads.cigar[reads.cigar_off[i]:reads.cigar_off[i + 1]]]
        lq = int(reads.seq_len[i])
        seq = bytes(reads.seq[reads.seq_off[i]:reads.seq_off[i] + (lq + 1) // 2])
        md = bytes(reads.md[reads.md_off[i]:reads.md_off[i + 1]]).decode()
        recs.append(Rec(0, int(reads.start[i]), f"u{i}", cigar=cig, seq=seq, l_seq=lq, aux=aux_Z("MD", md)))
    order = sorted(range(len(recs)), key=lambda i: (recs[i].pos, i))
    extra = [Rec(0, recs[order[0]].pos, "sec", flag=256, cigar=recs[order[0]].cigar, seq=recs[order[0]].seq,
                 l_seq=recs[order[0]].l_seq, aux=aux_Z("MD", "0"))]
    bam = str(tmp_path / "u.bam")
    write_bam(bam, [("chrU", 10_000_000)], extra + [recs[i] for i in order])
    vcf = tmp_path / "u.vcf"
    hdr = ["##fileformat=VCFv4.2", "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS"]
    vcf.write_text("\n".join(hdr + [f"chrU\t{p}\t.\t{r}\t{a}\t50\tPASS\t.\tGT\t{g}" for p, r, a, g in vrecs]) + "\n")
    return known, reads, order, bam, str(vcf)


def test_u_ingest_round_trip(tmp_path):
    import oracle
    from pomfret_amd.bam import BamFile, vcf_known_vars
    from pomfret_amd.synth_u import USpec
    known, reads, order, bam, vcf = _u_bam(tmp_path, USpec(n_reads=120, ref_len=200_000))
    kv = vcf_known_vars(vcf, "chrU")
    assert _kv_list(kv) == _kv_list(known)
    with BamFile(bam) as b:
        got, qn, info = b.fetch_contig_reads("chrU")
    assert info["n_truncated"] == 0
    with BamFile(bam, threads=5) as b:                   # BGZF inflate threads: the same reads
        got_t, qn_t, _ = b.fetch_contig_reads("chrU")
        got_t2, qn_t2, _ = b.fetch_contig_reads("chrU")
    assert qn_t == qn and qn_t2 == qn
    for f in ("start", "end", "cigar", "seq", "md"):
        assert np.array_equal(getattr(got_t, f), getattr(got, f)) and np.array_equal(getattr(got_t2, f), getattr(got, f))
    assert qn == [f"u{i}" for i in order]                 # the flag-256 record is skipped
    o = np.asarray(order)
    assert np.array_equal(got.start, reads.start[o]) and np.array_equal(got.end, reads.end[o])
    for k, i in enumerate(order):
        assert np.array_equal(got.md[got.md_off[k]:got.md_off[k + 1]], reads.md[reads.md_off[i]:reads.md_off[i + 1]])
    hp_f = oracle.haptag_reads(kv, got)
    hp_o = oracle.haptag_reads(known, reads)
    assert np.array_equal(hp_f, hp_o[o])


# ------------------------------------------------- f2 rescue of dropped sites
def _py_read_var_pos(pos0, cigar, md):
    """parse_variants_for_one_read (blockjoin.c:1545-1691), positions only."""
    out, ref = [], pos0
    for c in cigar:
        op, l = c & 15, c >> 4
        if op in (0, 2, 3, 7, 8):
            ref += l
        elif op == 1:
            out.append(ref)

    def ty(ch):
        if ch.isdigit():
            return 0
        if ch == "^":
            return 1
        return 2 if ch in "ATCGatcgUuNn" else 4
    ref, prev, pi = pos0, ty(md[0]), 0
    if prev == 2:
        out.append(ref)
        ref += 1
        prev = -1
    for i in range(1, len(md)):
        t = ty(md[i])
        if t == prev:
            continue
        if prev == 0:
            ref += int(md[pi:i])
        elif prev == 1:
            if t == 0:
                out.append(ref)
                ref += i - pi - 1
                prev, pi = t, i
            continue
        if t == 2:
            out.append(ref)
            ref += 1
            prev, pi = -1, i
        else:
            prev, pi = t, i
    return out


def _py_rescue(recs, known_pos, dropped, meth, raw=None):
    res, prev_i = {}, 0
    for s, e in dropped:
        start, end = (s - 1) & 0xFFFFFFFF, (e + 1) & 0xFFFFFFFF
        poss = []
        for i in range(prev_i, len(known_pos)):
            p = known_pos[i]
            if start <= p < end:
                poss.append(p)
            if p >= end:
                prev_i = i
                break
        if not poss:
            continue
        pb = [(p << 33) for p in poss]
        for j in expected_fetch(recs, recs[0].tid if recs else 0, start, end - 0, 0):
            r = recs[j]
            hm = meth.get(r.qname)
            if hm is None:
                continue
            if raw is not None:
                hr = raw.get(r.qname)
                if hr is None:
                    continue
            else:
                hr = 254
                if r.aux.startswith(b"HPi"):
                    v = int.from_bytes(r.aux[3:7], "little", signed=True)
                    hr = v - 1 if 1 <= v <= 255 else 254
            if hr == 254:
                continue
            md = r.aux[r.aux.index(b"MDZ") + 3:].split(b"\0")[0].decode()
            pb += [(p << 33) | (1 << 32) | hm for p in _py_read_var_pos(r.pos, r.cigar, md)]
        pb.sort()
        i = 0
        while i < len(pb) - 1:
            if pb[i] & (1 << 32):
                i += 1
                continue
            rp, c, j = pb[i] >> 33, [0, 0], i + 1
            while j < len(pb) and (pb[j] & (1 << 32)) and (pb[j] >> 33) == rp:
                h = pb[j] & 0xFF
                if h < 2:
                    c[h] += 1
                j += 1
            res[rp] = 1 if c[0] > c[1] else 0 if c[1] > c[0] else 254
            i = j
    return res


def test_rescue_dropped_matches_restatement(tmp_path):
    from pomfret_amd.abi import KnownVars
    from pomfret_amd.bam import BamFile, rescue_dropped
    rng = np.random.default_rng(4)
    seq = bytes([0x11] * 300)
    kpos = sorted(set(int(x) for x in rng.integers(1000, 20000, 60)))
    recs = []
    meth = {}
    for i in range(140):
        p = int(rng.integers(500, 19000))
        # a read of 600 bases with a mismatch / deletion / insertion at a known site or nearby
        k = kpos[int(rng.integers(0, len(kpos)))]
        off = k - p
        if not (10 <= off < 550):
            off = int(rng.integers(10, 500))
        kind = int(rng.integers(0, 3))
        if kind == 0:
            cig, md = [(600 << 4) | 0], f"{off}A{600 - off - 1}"
        elif kind == 1:
            cig, md = [(off << 4) | 0, (2 << 4) | 2, ((600 - off) << 4) | 0], f"{off}^AC{600 - off}"
        else:
            cig, md = [(off << 4) | 0, (3 << 4) | 1, ((597 - off) << 4) | 0], f"{597}"
        hp_tag = int(rng.integers(0, 3))                 # 0: HP absent -> unphased raw
        aux = (aux_i("HP", hp_tag) if hp_tag else b"") + aux_Z("MD", md)
        recs.append(Rec(0, p, f"q{i}", cigar=cig, seq=seq, l_seq=600, aux=aux))
        if rng.random() < 0.8:
            meth[f"q{i}"] = int(rng.integers(0, 3))
    recs.sort(key=lambda r: r.pos)
    p = str(tmp_path / "r.bam")
    write_bam(p, [("c", 100_000)], recs)
    kn = KnownVars(pos=np.array(kpos), len=np.ones(len(kpos)), op=np.ones(len(kpos)),
                   haptag=np.zeros(len(kpos)), char_off=np.arange(len(kpos) + 1), chars=np.zeros(len(kpos)))
    dropped = [(1200, 4000), (6000, 9000), (12000, 18000)]
    with BamFile(p) as b:
        got = rescue_dropped(b, "c", dropped, kn, meth)
        raw = {f"q{i}": int(rng.integers(0, 2)) for i in range(0, 140, 2)}
        got_raw = rescue_dropped(b, "c", dropped, kn, meth, raw)
    exp = _py_rescue(recs, kpos, dropped, meth)
    assert got == exp and len(got) > 5 and any(v != 254 for v in got.values())
    assert got_raw == _py_rescue(recs, kpos, dropped, meth, raw)
    # threads: the intervals spread over host threads give the serial result,
    # also with intervals that overlap (the last write per position wins and
    # the known-position cursor runs across the intervals in order)
    dropped2 = [(1200, 4000), (3000, 5200), (6000, 9000), (8800, 12500), (12000, 18000)]
    with BamFile(p) as b:
        for th in (2, 3, 8):
            assert rescue_dropped(b, "c", dropped, kn, meth, threads=th) == got
            assert rescue_dropped(b, "c", dropped, kn, meth, raw, threads=th) == got_raw
        one = rescue_dropped(b, "c", dropped2, kn, meth)
        assert rescue_dropped(b, "c", dropped2, kn, meth, threads=4) == one
    assert one == _py_rescue(recs, kpos, dropped2, meth)


def _py_cov(recs, lens):
    """estimate_read_coverage_dirtyfast (blockjoin.c:951-1040) restated."""
    covs = [0] * len(lens)
    prev, refid, bins = -1, -1, []
    for r in recs:
        refid = r.tid
        if refid < 0:
            continue
        if refid != prev:
            if prev >= 0:
                covs[prev] = sum(bins) // len(bins) if bins else 0
            bins = [0] * (lens[refid] // 5000)
            prev = refid
        if (r.flag & (4 | 256 | 2048)) or r.mapq < 5 or r.l_seq < 15000:
            continue
        de = -1.0
        if b"def" in r.aux:
            import struct
            k = r.aux.index(b"def")
            de = struct.unpack("<f", r.aux[k + 3:k + 7])[0]
        if de > 0.1:
            continue
        i, e = r.pos, endpos(r.pos, r.cigar, r.flag)
        while i < e:
            if i // 5000 < len(bins):
                bins[i // 5000] += 1
            i += 5000
    if refid >= 0:
        covs[refid] = sum(bins) // len(bins) if bins else 0
    return covs


def test_estimate_coverage(tmp_path):
    from pomfret_amd.bam import BamFile
    rng = np.random.default_rng(8)
    lens = [300_000, 123_456, 60_000]
    recs = []
    for tid in range(3):
        for _ in range(150 if tid < 2 else 60):
            L = int(rng.integers(5_000, 40_000))
            p = int(rng.integers(0, max(1, lens[tid] - 1000)))
            flag = int(rng.choice([0, 0, 0, 16, 256, 2048]))
            aux = aux_f("de", float(rng.choice([0.01, 0.05, 0.2]))) if rng.random() < 0.7 else b""
            recs.append(Rec(tid, p, f"t{tid}_{len(recs)}", flag=flag, mapq=int(rng.integers(0, 60)),
                            cigar=[(L << 4) | 0], seq=b"", l_seq=L, aux=aux))
    recs.sort(key=lambda r: (r.tid, r.pos))
    seqfix = []
    for r in recs:                                  # SEQ bytes sized to l_seq
        r.seq = bytes((r.l_seq + 1) // 2)
        seqfix.append(r)
    p1 = str(tmp_path / "cov.bam")
    write_bam(p1, [("a", lens[0]), ("b", lens[1]), ("c", lens[2])], seqfix)
    with BamFile(p1) as b:
        got = b.estimate_coverage()
        assert b.n_unplaced == 0
    assert got == _py_cov(seqfix, lens) and got[0] > 0
    # with BGZF inflate threads (bgzf_mt, the reference's -t N): the same pass
    for th in (2, 7):
        with BamFile(p1, threads=th) as b:
            assert b.estimate_coverage() == got
            assert b.estimate_coverage() == got            # a second pass seeks back: the ring restarts
    # an unplaced read at the end reassigns refID: the last contig keeps 0
    un = Rec(-1, -1, "unplaced", flag=4, cigar=[], seq=bytes(50), l_seq=100)
    p2 = str(tmp_path / "cov2.bam")
    write_bam(p2, [("a", lens[0]), ("b", lens[1]), ("c", lens[2])], seqfix + [un])
    with BamFile(p2) as b:
        got2 = b.estimate_coverage()
        assert b.n_unplaced == 1
    assert got2[:2] == got[:2] and got[2] > 0 and got2[2] == 0
