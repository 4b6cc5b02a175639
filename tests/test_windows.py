"""Window definition on the host, CPU only.

The product's pf_vcf_gaps (pomfret_amd/csrc/pf_windows.c) is checked against
the oracle's restatement (oracle/pf_oracle.c orc_vcf_gaps, pinned by the
reference's example fixture in test_oracle.py) on that fixture and on seeded
synthetic phased VCFs with the reference's quirks (multi-contig abs_start,
PS ".", unphased lines, revisited contigs, an unterminated last line).  The
reference's fatal exit for an unsorted POS is an error on the product side
only (the oracle logs and goes on); '#' lines are skipped unread, as
load_intervals_from_file does (blockjoin.c:2023-2026), so a multi-sample
#CHROM header only fails later, in the VCF writer.

pf_interval_gaps' GTF / TSV loader (--gtf / --tsv, insert_gtf_line
:1305-1345) is checked against the oracle's restatement on whatshap-shaped
GTFs and 3-column TSVs with the loader's quirks: per-contig abs_start, a
revisited contig continuing from the other contig's last end, comment lines,
runs of tabs, short lines, strtoul on odd numbers.

pf_report_windows is checked against a direct restatement of the
`pomfret report` chunk loop (blockjoin.c:4966-4980) in uint32 arithmetic.
"""
import gzip
import os
import random

import pytest

from pomfret_amd import _lib

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
HEADER = "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\n"


def _write(tmp_path, name, text, gz=True):
    p = os.path.join(tmp_path, name)
    if gz:
        with gzip.open(p, "wt") as f:
            f.write(text)
    else:
        with open(p, "w") as f:
            f.write(text)
    return p


def _line(ctg, pos, ps, fmt="GT:PS"):
    if fmt == "GT":
        return f"{ctg}\t{pos}\t.\tA\tC\t.\tPASS\t.\tGT\t0/1\n"
    return f"{ctg}\t{pos}\t.\tA\tC\t.\tPASS\t.\t{fmt}\t0|1:{ps}\n" if fmt == "GT:PS" else \
        f"{ctg}\t{pos}\t.\tA\tC\t.\tPASS\t.\t{fmt}\t{ps}:0|1:30\n"


def _synth_vcf(rng, n_contigs=3, revisit=False):
    """Phase blocks per contig; PS = first POS of the block (as WhatsHap
    writes it), with PS "." lines, unphased GT-only lines and a second FORMAT
    layout (PS first) mixed in."""
    lines = []
    per = {}
    names = [f"chr{i + 1}" for i in range(n_contigs)]
    order = names + ([names[0]] if revisit else [])
    for ctg in order:
        # a revisited contig continues above every POS seen so far: the
        # reference keeps prev_pos across a switch back (blockjoin.c:2042-2048)
        pos = max(per.values()) if ctg in per else rng.randrange(1, 200_000)
        for _ in range(rng.randrange(1, 8)):
            block0 = pos
            for j in range(rng.randrange(1, 30)):
                kind = rng.random()
                if kind < 0.08:
                    lines.append(_line(ctg, pos, ".", "GT:PS"))
                elif kind < 0.15:
                    lines.append(_line(ctg, pos, None, "GT"))
                elif kind < 0.25:
                    lines.append(_line(ctg, pos, block0, "PS:GT:GQ"))
                else:
                    lines.append(_line(ctg, pos, block0))
                pos += rng.randrange(1, 3000)
            pos += rng.choice([10, 1000, 30_000, 60_000, 200_000])
        per[ctg] = pos
    return HEADER + "".join(lines)


def test_example_fixture_matches_oracle(oracle_lib):
    p = os.path.join(GOLD, "example", "variants.vcf.gz")
    got = _lib.vcf_gaps(p)
    assert got == oracle_lib.vcf_gaps(p)
    assert got[0]["gaps"] == [(11092382, 11147866)]


@pytest.mark.parametrize("seed", range(12))
def test_synthetic_vcf_matches_oracle(oracle_lib, tmp_path, seed):
    rng = random.Random(seed)
    text = _synth_vcf(rng, n_contigs=1 + seed % 4, revisit=seed % 3 == 0)
    if seed % 5 == 4:
        text += "chrX\t5\t.\tA\tC\t.\tPASS\t.\tGT:PS\t0|1:5"       # no trailing newline: never parsed
    p = _write(str(tmp_path), "v.vcf.gz", text, gz=seed % 2 == 0)
    for readback in (0, 50_000):
        got = _lib.vcf_gaps(p, readback)
        want = oracle_lib.vcf_gaps(p, readback)
        assert got == want
    names = [c["name"] for c in got]
    assert "chrX" not in names
    # quirk kept from the reference: abs_start is only set on the first contig
    for c in got[1:]:
        assert c["abs_start"] == 0


def test_merge_threshold(oracle_lib, tmp_path):
    """Two raw gaps 100 bp apart merge at readback 50000 and stay apart at 50."""
    text = HEADER + "".join([
        _line("c", 100, 100), _line("c", 200, 100),
        _line("c", 5000, 5000), _line("c", 5100, 5000),
        _line("c", 6100, 6100), _line("c", 6200, 6100),
    ])
    p = _write(str(tmp_path), "m.vcf", text, gz=False)
    for rb in (50, 50_000):
        got = _lib.vcf_gaps(p, rb)
        assert got == oracle_lib.vcf_gaps(p, rb)
    assert _lib.vcf_gaps(p, 50_000)[0]["raw"] == [(200, 5000), (5100, 6100)]
    assert len(_lib.vcf_gaps(p, 50)[0]["gaps"]) == 2
    assert len(_lib.vcf_gaps(p, 50_000)[0]["gaps"]) == 1


def test_multi_sample_header_is_not_checked(oracle_lib, tmp_path):
    """the #CHROM column check of insert_vcf_line is never reached on the
    methphase path ('#' lines skipped first); the first sample column is read"""
    text = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\tS2\n" + \
        _line("c", 5, 5).rstrip("\n") + "\t0|1:9\n" + _line("c", 900, 900)
    p = _write(str(tmp_path), "b.vcf.gz", text)
    assert _lib.vcf_gaps(p) == oracle_lib.vcf_gaps(p)
    assert _lib.vcf_gaps(p)[0]["raw"] == [(5, 900)]


def _gtf_line(ctg, s, e):
    """whatshap stats --block-list GTF shape"""
    return f'{ctg}\tPhasing\texon\t{s}\t{e}\t.\t+\t.\tgene_id "{s}"; transcript_id "{s}.1";\n'


def _synth_blocks(rng, fmt, revisit=False):
    names = [f"chr{i + 1}" for i in range(rng.randrange(1, 4))]
    order = names + ([names[0]] if revisit else [])
    lines = ["# whatshap stats blocks\n"] if rng.random() < 0.5 else []
    for ctg in order:
        pos = rng.randrange(1, 300_000)
        for _ in range(rng.randrange(1, 9)):
            s = pos
            e = s + rng.randrange(1, 400_000)
            if fmt == 1:
                lines.append(_gtf_line(ctg, s, e))
            else:
                sep = "\t\t" if rng.random() < 0.1 else "\t"      # a run of tabs is one separator (strtok)
                lines.append(f"{ctg}{sep}{s}\t{e}\n")
            if rng.random() < 0.1:
                lines.append(f"{ctg}\n" if fmt == 2 else f"{ctg}\tPhasing\texon\n")   # short line
            pos = e + rng.choice([5, 2000, 30_000, 60_000, 250_000])
    return "".join(lines)


@pytest.mark.parametrize("seed", range(10))
def test_gtf_tsv_match_oracle(oracle_lib, tmp_path, seed):
    rng = random.Random(seed)
    fmt = 1 + seed % 2
    text = _synth_blocks(rng, fmt, revisit=seed % 3 == 0)
    if seed % 4 == 3:
        text += "chrZ\t5\t10" if fmt == 2 else _gtf_line("chrZ", 5, 10).rstrip("\n")   # never parsed
    p = _write(str(tmp_path), "b.gtf.gz" if fmt == 1 else "b.tsv", text, gz=seed % 2 == 0)
    for readback in (0, 50_000):
        got = _lib.interval_gaps(p, fmt, readback)
        assert got == oracle_lib.interval_gaps(p, fmt, readback)
    assert "chrZ" not in [c["name"] for c in got]


def test_gtf_quirks(oracle_lib, tmp_path):
    """hand-worked: gaps are [end of a block, start of the next]; every contig
    has its own abs_start (prev_end resets per new contig, :2098); a revisited
    contig continues from the other contig's last end; abs_end is set only when
    a NEW contig name follows (or at EOF, for the contig being read): b is
    left behind by a switch back to a, so its abs_end stays 0."""
    text = (_gtf_line("a", 100, 1000) + _gtf_line("a", 5000, 9000) + _gtf_line("b", 700, 800) +
            _gtf_line("b", 900, 1000) + _gtf_line("a", 20000, 30000))
    p = _write(str(tmp_path), "q.gtf", text, gz=False)
    got = _lib.interval_gaps(p, _lib.INTERVALS_GTF, 50)
    assert got == oracle_lib.interval_gaps(p, 1, 50)
    a, b = got
    assert (a["abs_start"], b["abs_start"]) == (100, 700)
    assert a["raw"] == [(1000, 5000), (1000, 20000)]          # the revisit's gap starts at b's last end
    assert b["raw"] == [(800, 900)]
    assert (a["abs_end"], b["abs_end"]) == (30000, 0)
    tsv = _write(str(tmp_path), "q.tsv", "a\t+10\t-5\na\t 20\t99999999999999999999999\na\t30\t40\n", gz=False)
    t, = _lib.interval_gaps(tsv, _lib.INTERVALS_TSV, 0)
    assert t == oracle_lib.interval_gaps(tsv, 2, 0)[0]
    # strtoul: '-' negates; an overflow saturates to UINT32_MAX, which is the
    # "no block yet" marker, so the next start is taken as abs_start again
    assert t["raw"] == [(2**32 - 5, 20)] and t["abs_start"] == 30


def test_empty_and_header_only(tmp_path):
    p = _write(str(tmp_path), "h.vcf.gz", HEADER)
    assert _lib.vcf_gaps(p) == []


def test_fatal_cases_are_errors(tmp_path):
    unsorted = HEADER + _line("c", 500, 500) + _line("c", 400, 500)
    p = _write(str(tmp_path), "u.vcf.gz", unsorted)
    with pytest.raises(_lib.PomfretError):
        _lib.vcf_gaps(p)
    with pytest.raises(_lib.PomfretError):
        _lib.vcf_gaps(os.path.join(str(tmp_path), "missing.vcf.gz"))
    # switching back to a contig keeps the last contig's prev_pos, so a lower
    # POS there is "not sorted" (blockjoin.c:1383-1387 after :2042-2048)
    revisit = HEADER + _line("a", 900, 900) + _line("b", 50, 50) + _line("b", 70_000, 70_000) + \
        _line("a", 1000, 900)
    p = _write(str(tmp_path), "r.vcf.gz", revisit)
    with pytest.raises(_lib.PomfretError):
        _lib.vcf_gaps(p)


# --------------------------------------------------------------------------
# pomfret report chunk windows (a14)
def _report_windows_ref(abs_start, gaps, chunk_size, chunk_stride):
    """blockjoin.c:4966-4980 with uint32 wrap-around."""
    M = 0xFFFFFFFF
    out = []
    prev = abs_start
    for start, end in gaps:
        if ((start - prev) & M) > chunk_size:
            i = prev
            while ((i + chunk_stride) & M) < start:
                out.append((i, (i + chunk_size) & M))
                i = (i + chunk_stride) & M
        prev = end
    return out


def test_report_windows_example(oracle_lib):
    c = _lib.vcf_gaps(os.path.join(GOLD, "example", "variants.vcf.gz"))[0]
    got = _lib.report_windows(c["abs_start"], c["raw"], 2000, 1000)
    assert got == _report_windows_ref(c["abs_start"], c["raw"], 2000, 1000)
    assert got[0] == (c["abs_start"], c["abs_start"] + 2000)
    assert len(got) == (11092382 - 11082691 - 1) // 1000


@pytest.mark.parametrize("seed", range(8))
def test_report_windows_random(seed):
    rng = random.Random(seed)
    abs_start = rng.randrange(0, 1_000_000)
    gaps, pos = [], abs_start
    for _ in range(rng.randrange(0, 20)):
        s = pos + rng.randrange(0, 300_000)
        e = s + rng.randrange(1, 80_000)
        if rng.random() < 0.1:
            s, e = e, s          # out-of-order raw gap: uint32 arithmetic wraps
        gaps.append((s, e))
        pos = max(s, e)
    cs, st = rng.choice([(50_000, 25_000), (10_000, 10_000), (2000, 3000)])
    got = _lib.report_windows(abs_start, gaps, cs, st)
    assert got == _report_windows_ref(abs_start, gaps, cs, st)


def test_report_windows_empty():
    assert _lib.report_windows(100, [], 1000, 500) == []
